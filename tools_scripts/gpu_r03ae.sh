#!/bin/bash
# Round 3, call ae: the N>1 launch rehearsed on one GPU (CPD_BENCH_SHARE_GPU=1:
# both ranks on GPU 0, harness collectives over gloo, 4096-row batches), with
# the end-to-end worker leg (one make_cpd_auto per rank) — plumbing only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CPD_BENCH_SHARE_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-pmc \
    > gpurun_out/r03ae_share2.json 2> gpurun_out/r03ae_share2.err \
    || { echo "2-rank rehearsal failed"; tail -30 gpurun_out/r03ae_share2.err; exit 1; }
python -c "
import json
d = json.loads(open('gpurun_out/r03ae_share2.json').read().strip().splitlines()[-1])
fb = d.get('full_build') or {}
print('2 ranks (shared GPU, rehearsal only):', d['n_gpus'], d['value'], d['config']['rows_per_step_per_gpu'],
      'full_build', fb.get('total_s'), fb.get('rows'), fb.get('what', '')[:60])"
