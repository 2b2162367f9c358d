#!/bin/bash
# Round 3, call ac: the HBM reserve of the auto batch (library and
# make_cpd_auto --hbm-reserve), with the parity and driver suites.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_hbm_reserve.py tests/test_gpu_drivers.py tests/test_gpu_parity.py \
    -x -v --timeout 200 --timeout-method thread > gpurun_out/r03ac_tests.log 2>&1 \
    || { echo "TESTS FAILED"; tail -40 gpurun_out/r03ac_tests.log; exit 1; }
tail -2 gpurun_out/r03ac_tests.log
