#!/bin/bash
# One GPU call on the current tree: the full -m gpu suite, the driver's default
# bench line, and a rocprofv3 kernel-trace --stats of the same workload.
#   tools_scripts/gpu_r02_final.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r02b}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
      > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/${TAG}_gputest.log; exit 1; }
  tail -3 gpurun_out/${TAG}_gputest.log
fi
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG --output-format csv \
    -- python3 $R/bench.py --no-pmc --no-cpu > $R/gpurun_out/prof_${TAG}_bench.json 2> $R/gpurun_out/prof_${TAG}_bench.err \
    || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_${TAG}_bench.err; exit 1; }
echo prof-done
