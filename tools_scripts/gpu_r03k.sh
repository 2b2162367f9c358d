#!/bin/bash
# Round 3, call k: GPU contraction with the wave-cooperative searches:
# identity tests, then 1M timing under three wave thresholds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ch_gpu.py -x -v -s --timeout 500 --timeout-method thread \
    > gpurun_out/r03k_ch_gpu.log 2>&1 || { echo "CH TESTS FAILED"; tail -40 gpurun_out/r03k_ch_gpu.log; exit 1; }
grep -E "passed|failed|1M CH" gpurun_out/r03k_ch_gpu.log
for wv in 8192; do for cap in 100000; do
  CPD_CH_LANE_CAP=$cap CPD_CH_WAVE=$wv timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03k_time_${wv}_$cap.log 2>&1 || { echo "timing $wv failed"; tail -5 gpurun_out/r03k_time_${wv}_$cap.log; exit 1; }
  echo "wave_max=$wv cap=$cap"; grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03k_time_${wv}_$cap.log
done; done
