#!/bin/bash
# Round 3, call y: the end-to-end worker's D2H export against the number of
# writer threads (div 8 worker 0 of the 1M graph, --discard, warm plan).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
T=$(mktemp -d /tmp/cpde2e.XXXX)
trap 'rm -rf $T' EXIT
timeout -k 10 120 $R/bin/gen_synth --width 1000 --height 1000 --seed 1 --out $T/g > /dev/null || exit 1
A="--input $T/g.xy --partmethod div --partkey 8 --workerid 0 --maxworker 8 --device 0 --outdir $T/out --discard --plan $T/g.plan"
mkdir -p $T/out
timeout -k 10 120 $R/bin/make_cpd_auto $A --plan-only > /dev/null || exit 1
for wt in 4 8 16 24; do
  timeout -k 10 300 $R/bin/make_cpd_auto $A --write-threads $wt > $O/r03y_wt$wt.log 2>&1 || { echo "e2e wt=$wt failed"; tail -5 $O/r03y_wt$wt.log; exit 1; }
  echo "wt=$wt: $(grep make_cpd_auto-json $O/r03y_wt$wt.log)"
done
