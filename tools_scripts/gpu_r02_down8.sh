#!/bin/bash
# Down-sweep A/B: column-major narrow bases (all K) and K slots per wave.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CPD_DOWN8_K=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r02_down8_k4_tests.log 2>&1 || { echo "K=4 TESTS FAILED"; tail -30 gpurun_out/r02_down8_k4_tests.log; exit 1; }
tail -2 gpurun_out/r02_down8_k4_tests.log
for k in 1 2 4 8 1; do
  CPD_DOWN8_K=$k timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-pmc --no-cpu --queries 200000 \
     > gpurun_out/r02_down8_k$k.json 2> gpurun_out/r02_down8_k$k.err || { echo "bench K=$k failed"; tail -20 gpurun_out/r02_down8_k$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_down8_k$k.json'));k=d['kernels'];print('K=$k', d['value'], 'down', k['sweep_down']['ms']/10, 'fm', k['first_moves']['ms']/10, 'frac', d['roofline']['frac'])"
done
