#!/bin/bash
# Round 3, call i: the early up-sweep's leaf-form init as a small grid-stride
# kernel (CPD_UP_INIT_BLOCKS) against one block per row (the old grid), then a
# kernel trace of the default for the step timeline.
set -o pipefail
TAG=${1:-r03i}
R=$PWD
bash tools_scripts/gpu_ab_env.sh $TAG CPD_UP_INIT_BLOCKS "512 1000000000 2048" \
    "tests/test_gpu_parity.py tests/test_gpu_switches.py" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_$TAG --output-format csv \
    -- python3 $R/bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 4 --queries 1000 > $R/gpurun_out/trace_${TAG}.json 2> $R/gpurun_out/trace_${TAG}.err \
    || { echo "trace failed"; tail -5 $R/gpurun_out/trace_${TAG}.err; exit 1; }
echo trace-done
