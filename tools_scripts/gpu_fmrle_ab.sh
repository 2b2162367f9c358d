#!/bin/bash
# Fused first-moves + RLE count: GPU parity (rows bit-exact vs the oracle at
# small and at BASELINE sizes), then the bench A/B over CPD_FM_RLE
# (0 = first_moves_n4 + rle_count; 16 / 32 / 64 segments per chunk).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fmrle}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
    || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for v in ${FMRLE_VALUES:-32 0 16 64}; do
  CPD_FM_RLE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search \
      --queries 100000 > gpurun_out/${TAG}_b$v.json 2> gpurun_out/${TAG}_b$v.err \
      || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_b$v.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_b$v.json'));k=d['kernels'];print('FM_RLE=$v', d['value'], d['ms_per_step'], d['parity_sample_bit_exact'], {n:round(v['ms']/v['launches'],3) for n,v in k.items()})"
done
