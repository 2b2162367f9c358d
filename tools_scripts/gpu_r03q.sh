#!/bin/bash
# Round 3, call q: expand_rows rewrite (run-owned words, 4 chunks per wave):
# index/parity tests, then kernel stats of a short bench (its index build
# expands the last batch's 21504 rows).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_index_stream.py tests/test_gpu_parity.py tests/test_gpu_drivers.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03q_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03q_tests.log; exit 1; }
tail -2 gpurun_out/r03q_tests.log
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03q --output-format csv \
    -- python3 $R/bench.py --no-pmc --no-cpu --no-full-build --no-search --steps 3 > $R/gpurun_out/prof_r03q_bench.json 2> $R/gpurun_out/prof_r03q_bench.err \
    || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_r03q_bench.err; exit 1; }
grep -h -E "expand_rows|validate_rows|table_walk" $R/gpurun_out/prof_r03q/*/*kernel_stats.csv | cut -c1-60,200-400
