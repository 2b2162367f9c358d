#!/bin/bash
# Round 3, call n: GPU contraction stage timings at 1M, then a short bench
# with the end-to-end worker build (GPU-contracted plan).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03n_ch_time.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r03n_ch_time.log; exit 1; }
grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03n_ch_time.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --queries 200000 \
    > gpurun_out/r03n_bench.json 2> gpurun_out/r03n_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03n_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r03n_bench.json'));print(d['value'], d['ms_per_step'], d['hierarchy'], json.dumps(d.get('full_build')))"
