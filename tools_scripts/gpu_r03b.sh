#!/bin/bash
# Round 3, call b: index tests (new expand/validate kernels), the bench with
# query timings, the walk's L2/fabric counters and the gather microbenchmark.
set -o pipefail
TAG=${1:-r03b}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 700 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_index_stream.py tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_drivers.py tests/test_gpu_switches.py tests/test_gpu_melb_standin.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
timeout -k 10 600 python bench.py --no-cpu --no-full-build > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['ms_per_step'],d['queries_per_s'],d['pmc_traffic_per_launch'].get('expand_rows'))"
timeout -k 10 600 python3 tools_scripts/walk_pmc.py gpurun_out/${TAG}_walk_pmc.json > gpurun_out/${TAG}_walk_pmc.log 2>&1 \
    || { echo "walk pmc failed"; tail -20 gpurun_out/${TAG}_walk_pmc.log; exit 1; }
echo walk-pmc-done
timeout -k 10 300 tools_scripts/bin/gather_ceiling 10 512 > gpurun_out/${TAG}_gather_ceiling.json 2>&1 \
    || { echo "gather failed"; cat gpurun_out/${TAG}_gather_ceiling.json; exit 1; }
cat gpurun_out/${TAG}_gather_ceiling.json
