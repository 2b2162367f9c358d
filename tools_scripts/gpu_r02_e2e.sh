#!/bin/bash
# End-to-end worker build at the north-star size: the 1M-node graph, one
# worker's buckets (div 64, worker 0 of 64: 15,625 rows ~ 39 GB of RLE
# buckets), make_cpd_auto's own timing line (CH, GPU build, export + write),
# then fifo_auto streaming those buckets into its index and one query batch
# through the reference's FIFO protocol.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W=/tmp/e2e; rm -rf $W; mkdir -p $W
df -h /tmp $GRAFT_REPO_ROOT | tee gpurun_out/r02_e2e_df.txt
free -g | tee -a gpurun_out/r02_e2e_df.txt
timeout -k 10 120 bin/gen_synth --width 1000 --seed 1 --out $W/synth1m --queries 20000 > gpurun_out/r02_e2e.log 2>&1 || exit 1
AV=$(df --output=avail -k /tmp | tail -n1)
EXTRA=""
if [ "$AV" -lt 50000000 ]; then EXTRA="--targets-from $W/synth1m.scen"; echo "disk < 120 GB: rows of the scenario's targets only" | tee -a gpurun_out/r02_e2e.log; fi
timeout -k 10 600 bin/make_cpd_auto --input $W/synth1m.xy --partmethod div --partkey 64 --workerid 0 --maxworker 64 --outdir $W/index $EXTRA >> gpurun_out/r02_e2e.log 2>&1 || { tail -5 gpurun_out/r02_e2e.log; exit 1; }
du -sh $W/index | tee -a gpurun_out/r02_e2e.log
# second worker start with the plan cached (what the other 63 workers see)
timeout -k 10 600 bin/make_cpd_auto --input $W/synth1m.xy --partmethod div --partkey 64 --workerid 1 --maxworker 64 --outdir $W/index1 --plan $(ls $W/index/*.plan) --targets-from $W/synth1m.scen >> gpurun_out/r02_e2e.log 2>&1 || { tail -5 gpurun_out/r02_e2e.log; exit 1; }
rm -rf $W/index1
timeout -k 10 300 bin/fifo_auto --input $W/synth1m.xy $W/synth1m.xy.diff --partmethod div --partkey 64 --workerid 0 --maxworker 64 --outdir $W/index --alg table-search --fifo $W/w0.fifo --once >> gpurun_out/r02_e2e.log 2>&1 &
FP=$!
for i in $(seq 1 240); do grep -q listening gpurun_out/r02_e2e.log && break; sleep 1; done
python - <<PY >> gpurun_out/r02_e2e.log 2>&1
import numpy as np, os
q = [l.split()[1:] for l in open("$W/synth1m.scen") if l.startswith("q")]
n = 1000000; chunk = -(-n // 64)
mine = [(int(s), int(t)) for s, t in q if (int(t) // chunk) % 64 == 0]
mine = mine[:5000] if mine else []
if not mine:  # the full worker: its own targets
    rng = np.random.default_rng(2)
    mine = [(int(rng.integers(0, n)), int(t)) for t in rng.integers(0, chunk, 50000)]
open("$W/q0", "w").write(f"{len(mine)}\n" + "".join(f"{s} {t}\n" for s, t in mine))
os.mkfifo("$W/a0")
with open("$W/w0.fifo", "w") as f:
    f.write('{"hscale": 1.0, "fscale": 0.0, "time": 0, "itrs": -1, "k_moves": -1, "threads": 0, "verbose": false, "debug": false, "thread_alloc": false, "no_cache": false}\n$W/q0 $W/a0 -\n')
print("queries", len(mine), "answer:", open("$W/a0").read().strip())
PY
wait $FP
cat gpurun_out/r02_e2e.log | grep -v "^$"
rm -rf $W
