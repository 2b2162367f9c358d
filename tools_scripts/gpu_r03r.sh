#!/bin/bash
# Round 3, call r: GPU contraction with small/large LDS wave searches
# (identity tests + 1M timing), expand_rows segmented fill (index tests +
# kernel time at 1 and 4 chunks per wave).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
bash tools_scripts/gpu_r03k.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_index_stream.py tests/test_gpu_drivers.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03r_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03r_tests.log; exit 1; }
tail -2 gpurun_out/r03r_tests.log
cd /tmp
for cpw in 1 4 16; do
  CPD_EXP_CPW=$cpw timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03r_$cpw --output-format csv \
      -- python3 $R/bench.py --no-pmc --no-cpu --no-full-build --no-search --steps 3 > $R/gpurun_out/prof_r03r_$cpw.json 2> $R/gpurun_out/prof_r03r_$cpw.err \
      || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_r03r_$cpw.err; exit 1; }
  echo "cpw=$cpw"; grep -h "expand_rows" $R/gpurun_out/prof_r03r_$cpw/*/*kernel_stats.csv | cut -d, -f2-4
done
