#!/bin/bash
# End-to-end make_cpd_auto worker (configs[3]: 1M-node graph, div 8, worker 0,
# cold plan cache, DOSCPD02 files written) under several batch widths and
# writer-thread counts: one JSON phase line per setting.
#   tools_scripts/e2e_worker_sweep.sh TAG "B:T B:T ..."
set -o pipefail
TAG=${1:-e2e}
CFGS=${2:-"4096:8 4096:16 8192:16 0:16"}
R=$PWD
W=/tmp/cpd-e2e-sweep
mkdir -p $W gpurun_out
[ -f $W/g.xy ] || $R/bin/gen_synth --width 1000 --seed 1 --style shuffled --out $W/g > /dev/null || exit 1
for c in $CFGS; do
  B=${c%%:*}; T=${c#*:}
  rm -rf $W/out; mkdir -p $W/out
  timeout -k 10 300 env ${ENVS:-} $R/bin/make_cpd_auto --input $W/g.xy --partmethod div --partkey 8 --workerid 0 \
      --maxworker 8 --outdir $W/out --device 0 --batch $B --write-threads $T > $W/log 2>&1 \
      || { echo "make_cpd_auto B=$B T=$T failed"; tail -5 $W/log; exit 1; }
  echo "B=$B T=$T $(grep make_cpd_auto-json $W/log)" | tee -a $R/gpurun_out/${TAG}_e2e.log
  du -sh $W/out | tee -a $R/gpurun_out/${TAG}_e2e.log
done
rm -rf $W/out
