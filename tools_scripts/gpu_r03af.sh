#!/bin/bash
# Round 3, call af: GPU contraction with the wave heap written by lane 0 alone;
# identity tests (every route, make_cpd_auto files), 1M timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ch_gpu.py -x -v -s --timeout 500 --timeout-method thread \
    > gpurun_out/r03af_ch_gpu.log 2>&1 || { echo "CH TESTS FAILED"; tail -40 gpurun_out/r03af_ch_gpu.log; exit 1; }
grep -E "passed|failed|1M CH" gpurun_out/r03af_ch_gpu.log
timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03af_time.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r03af_time.log; exit 1; }
grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03af_time.log | tail -2
timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03af_time2.log 2>&1 && grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03af_time2.log | tail -2
