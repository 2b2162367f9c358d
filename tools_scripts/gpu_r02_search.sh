#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r02_search_tests.log 2>&1 || { echo "SEARCH TESTS FAILED"; tail -40 gpurun_out/r02_search_tests.log; exit 1; }
tail -3 gpurun_out/r02_search_tests.log
