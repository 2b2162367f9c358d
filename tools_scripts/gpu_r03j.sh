#!/bin/bash
# Round 3, call j: GPU contraction vs the host build (identical hierarchy,
# 1M timing), then the step-timeline trace of the default bench.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ch_gpu.py -x -v -s --timeout 500 --timeout-method thread \
    > gpurun_out/r03j_ch_gpu.log 2>&1 || { echo "CH TESTS FAILED"; tail -40 gpurun_out/r03j_ch_gpu.log; exit 1; }
tail -5 gpurun_out/r03j_ch_gpu.log; grep "1M CH" gpurun_out/r03j_ch_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_r03j --output-format csv \
    -- python3 $R/bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 4 --queries 1000 > $R/gpurun_out/trace_r03j.json 2> $R/gpurun_out/trace_r03j.err \
    || { echo "trace failed"; tail -5 $R/gpurun_out/trace_r03j.err; exit 1; }
echo trace-done
