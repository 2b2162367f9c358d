#!/bin/bash
# Round 3, call p: make_cpd_auto end to end (div 8 worker 0 of the 1M
# graph, --discard), GPU-contracted plan vs the host build's, with the
# per-batch host trace; then the split-up-sweep A/B (gpu_r03o.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
T=$(mktemp -d /tmp/cpde2e.XXXX)
trap 'rm -rf $T' EXIT
timeout -k 10 120 $R/bin/gen_synth --width 1000 --height 1000 --seed 1 --out $T/g > /dev/null || exit 1
for mode in gpu host gpu; do
  rm -rf $T/out; mkdir -p $T/out
  extra=""; [ $mode = host ] && extra="--ch-host"
  CPD_TRACE=1 timeout -k 10 300 $R/bin/make_cpd_auto --input $T/g.xy --partmethod div --partkey 8 --workerid 0 --maxworker 8 \
      --device 0 --outdir $T/out --discard --no-plan-cache $extra > $O/r03p_e2e_$mode.log 2>&1 || { echo "e2e $mode failed"; tail -5 $O/r03p_e2e_$mode.log; exit 1; }
  echo "$mode: $(grep make_cpd_auto-json $O/r03p_e2e_$mode.log)"
done
