#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench workload (no PMC child, no
# CPU legs, no end-to-end worker): the per-kernel averages the bench line's
# roofline is checked against.   tools_scripts/prof_round.sh TAG
set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${1:-round} --output-format csv \
  -- python3 $R/bench.py --no-pmc --no-cpu --no-full-build > $R/gpurun_out/prof_${1:-round}_bench.json 2> $R/gpurun_out/prof_${1:-round}_bench.err \
  || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_${1:-round}_bench.err; exit 1; }
echo prof-done
