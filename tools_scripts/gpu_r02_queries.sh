#!/bin/bash
# Round 2, first GPU check: full -m gpu suite, then the query kernels A/B
# (v2 = co-fetch + lane refill + ILP, v1 = lane per query) on the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r02_gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/r02_gputest.log; exit 1; }
tail -3 gpurun_out/r02_gputest.log
for v in 0 1; do
  CPD_TS_V1=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-pmc --no-cpu \
      > gpurun_out/r02_bench_tsv1_$v.json 2> gpurun_out/r02_bench_tsv1_$v.err || { echo "bench v1=$v failed"; tail -20 gpurun_out/r02_bench_tsv1_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_bench_tsv1_$v.json'));print('v1=$v', d['value'], d['queries_per_s'], d['queries_per_s_rle'], d['queries_per_s_congested'])"
done
