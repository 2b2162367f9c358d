#!/bin/bash
# Round 3, call ab: a 6.6-KB wave stage for simulation searches
# (CPD_CH_MICRO=1): identity tests with it on, 1M timing on and off.
set -o pipefail
mkdir -p gpurun_out
CPD_CH_MICRO=1 timeout -k 10 600 python -u -m pytest tests/test_ch_gpu.py -x -v -s --timeout 500 --timeout-method thread \
    > gpurun_out/r03ab_ch_gpu.log 2>&1 || { echo "CH TESTS FAILED"; tail -40 gpurun_out/r03ab_ch_gpu.log; exit 1; }
grep -E "passed|failed|1M CH" gpurun_out/r03ab_ch_gpu.log
for m in 1 0 1 0; do
  CPD_CH_MICRO=$m timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03ab_time_micro$m.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r03ab_time_micro$m.log; exit 1; }
  echo "micro=$m"; grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03ab_time_micro$m.log | tail -2
done
