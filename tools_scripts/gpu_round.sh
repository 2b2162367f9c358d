#!/bin/bash
# One GPU call on the current tree: the full -m gpu suite, smoke(), the
# driver's default bench line (with the end-to-end worker build), and a
# rocprofv3 kernel-trace --stats of the bench workload.
#   tools_scripts/gpu_round.sh TAG [skip-tests] [skip-prof]
set -o pipefail
TAG=${1:-round}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=20 \
      > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/${TAG}_gputest.log; exit 1; }
  tail -3 gpurun_out/${TAG}_gputest.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 700 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
if [ "$3" != "skip-prof" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG --output-format csv \
      -- python3 $R/bench.py --no-pmc --no-cpu --no-full-build > $R/gpurun_out/prof_${TAG}_bench.json 2> $R/gpurun_out/prof_${TAG}_bench.err \
      || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_${TAG}_bench.err; exit 1; }
  echo prof-done
fi
