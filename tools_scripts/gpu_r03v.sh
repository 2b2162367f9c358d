#!/bin/bash
# Round 3, call v: expand_rows with the bitmap run lookup: index / driver /
# parity tests, kernel time; then the contraction-priority A/B (gpu_r03u.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_index_stream.py tests/test_gpu_drivers.py tests/test_gpu_parity.py tests/test_ch_gpu.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03v_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03v_tests.log; exit 1; }
tail -2 gpurun_out/r03v_tests.log
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03v --output-format csv \
    -- python3 $R/bench.py --no-pmc --no-cpu --no-full-build --no-search --steps 3 > $R/gpurun_out/prof_r03v.json 2> $R/gpurun_out/prof_r03v.err \
    || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_r03v.err; exit 1; }
grep -h "expand_rows" $R/gpurun_out/prof_r03v/*/*kernel_stats.csv | python3 -c "
import sys,csv
for r in csv.reader(sys.stdin): print('expand_rows calls', r[1], 'avg_us %.1f' % (float(r[3]) / 1e3))"
python3 -c "import json;d=json.load(open('$R/gpurun_out/prof_r03v.json'));print('parity', d['parity_sample_bit_exact'], d['queries_per_s'])"
cd $R && bash tools_scripts/gpu_r03u.sh
cd $R
for t in 0 1; do
  CPD_CH_TINY=$t timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03v_time_tiny$t.log 2>&1 || { echo "timing tiny=$t failed"; exit 1; }
  echo "tiny=$t"; grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03v_time_tiny$t.log | tail -2
done
