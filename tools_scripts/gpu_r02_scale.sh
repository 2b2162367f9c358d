#!/bin/bash
# Full -m gpu suite (now with the at-size modules), then one quick bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
    > gpurun_out/r02_gputest_scale.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/r02_gputest_scale.log; exit 1; }
tail -22 gpurun_out/r02_gputest_scale.log
