#!/bin/bash
# Step timelines: a rocprofv3 kernel trace of a short build-only bench run
# per batch width, then tools_scripts/step_timeline.py on a steady step.
#   tools_scripts/trace_steps.sh TAG "28672 24576" [extra bench args]
set -o pipefail
TAG=$1; BATCHES=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for b in $BATCHES; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_${TAG}_b$b \
      -- python3 $R/bench.py --steps 8 --warmup 2 --batch $b --no-cpu --no-pmc --no-search \
         --no-full-build --queries 100000 "$@" > $R/gpurun_out/tr_${TAG}_b$b.json 2> $R/gpurun_out/tr_${TAG}_b$b.err ) \
      || { echo "trace $b failed"; tail -20 gpurun_out/tr_${TAG}_b$b.err; exit 1; }
  # the bench process's trace (the plan-building child writes its own)
  f=$(python3 -c "import glob,sys;fs=glob.glob('gpurun_out/tr_${TAG}_b$b/**/*kernel_trace.csv',recursive=True);print(max(fs,key=lambda x:open(x).read().count('first_moves')))")
  python3 tools_scripts/step_timeline.py "$f" > gpurun_out/tr_${TAG}_b${b}_timeline.txt
  python3 -c "import json;d=json.load(open('gpurun_out/tr_${TAG}_b$b.json'));print('b=$b', d['value'], d['ms_per_step'])"
  cat gpurun_out/tr_${TAG}_b${b}_timeline.txt
  rm -rf gpurun_out/tr_${TAG}_b$b
done
