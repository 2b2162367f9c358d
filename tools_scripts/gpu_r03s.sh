#!/bin/bash
# Round 3, call s: GPU contraction wave thresholds at 1M; expand_rows (lane
# per word, several chunks per wave) tests + kernel time per chunks-per-wave.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for wv in 16384 32768 65536; do
  CPD_CH_WAVE=$wv timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03s_time_$wv.log 2>&1 || { echo "timing $wv failed"; tail -5 gpurun_out/r03s_time_$wv.log; exit 1; }
  echo "wave_max=$wv"; grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03s_time_$wv.log | tail -2
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_index_stream.py tests/test_gpu_drivers.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03s_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03s_tests.log; exit 1; }
tail -2 gpurun_out/r03s_tests.log
cd /tmp
for cpw in 1 4 16; do
  CPD_EXP_CPW=$cpw timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03s_$cpw --output-format csv \
      -- python3 $R/bench.py --no-pmc --no-cpu --no-full-build --no-search --steps 3 > $R/gpurun_out/prof_r03s_$cpw.json 2> $R/gpurun_out/prof_r03s_$cpw.err \
      || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_r03s_$cpw.err; exit 1; }
  grep -h "expand_rows" $R/gpurun_out/prof_r03s_$cpw/*/*kernel_stats.csv | python3 -c "
import sys,csv
for r in csv.reader(sys.stdin): print('cpw=$cpw expand_rows calls', r[1], 'avg_us %.1f' % (float(r[3]) / 1e3))"
done
