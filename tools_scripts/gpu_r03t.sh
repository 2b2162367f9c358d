#!/bin/bash
# Round 3, call t: wave searches carrying each heap entry's list (one global
# round trip less per settled node): identity tests, then 1M timing per
# wave threshold.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ch_gpu.py -x -v -s --timeout 500 --timeout-method thread \
    > gpurun_out/r03t_ch_gpu.log 2>&1 || { echo "CH TESTS FAILED"; tail -40 gpurun_out/r03t_ch_gpu.log; exit 1; }
grep -E "passed|failed|1M CH" gpurun_out/r03t_ch_gpu.log
for wv in 65536 262144 1000000000; do
  CPD_CH_WAVE=$wv timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03t_time_$wv.log 2>&1 || { echo "timing $wv failed"; tail -5 gpurun_out/r03t_time_$wv.log; exit 1; }
  echo "wave_max=$wv"; grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03t_time_$wv.log | tail -2
done
