#!/bin/bash
# Full -m gpu suite, the driver's default bench command, per-level PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=10 \
    > gpurun_out/r02_gputest_all.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/r02_gputest_all.log; exit 1; }
tail -3 gpurun_out/r02_gputest_all.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err \
    || { echo "bench failed"; tail -20 gpurun_out/r02_bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02_bench_default.json'));print(d['value'], d['queries_per_s'], d['cpu_baseline']['value'], d['parity_sample_bit_exact'], json.dumps(d['cpd_search']))"
bash tools_scripts/gpu_r02_levels.sh
