#!/bin/bash
# first_moves write-amplification A/B: CPD_FM_X = segments exchanged per
# workgroup (1 = 16-B stores, 2 = 32 B, 4 = 64 B contiguous per row).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CPD_FM_X=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r02_fmx4_tests.log 2>&1 || { echo "X=4 TESTS FAILED"; tail -30 gpurun_out/r02_fmx4_tests.log; exit 1; }
CPD_FM_X=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r02_fmx2_tests.log 2>&1 || { echo "X=2 TESTS FAILED"; tail -30 gpurun_out/r02_fmx2_tests.log; exit 1; }
tail -n1 gpurun_out/r02_fmx4_tests.log; tail -n1 gpurun_out/r02_fmx2_tests.log
for x in 4 2 1; do
  CPD_FM_X=$x timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --queries 200000 \
     > gpurun_out/r02_fmx$x.json 2> gpurun_out/r02_fmx$x.err || { echo "bench X=$x failed"; tail -20 gpurun_out/r02_fmx$x.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_fmx$x.json'));k=d['kernels'];p=d['pmc_traffic_per_launch']['first_moves'];print('X=$x', d['value'], 'down', round(k['sweep_down']['ms']/10,2), 'fm', round(k['first_moves']['ms']/10,2), 'fm PMC read', p['read']/1e9, 'write', p['write']/1e9)"
done
