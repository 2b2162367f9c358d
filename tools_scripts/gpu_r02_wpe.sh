#!/bin/bash
# narrow down-sweep occupancy A/B: CPD_DOWN8_WPE = waves per SIMD asked of
# the compiler (1 = none: 88 VGPRs, 5 waves; 6 = 80 VGPRs, 6 waves, spills)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r02_wpe_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r02_wpe_tests.log; exit 1; }
CPD_DOWN8_WPE=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r02_wpe6_tests.log 2>&1 || { echo "WPE6 TESTS FAILED"; tail -30 gpurun_out/r02_wpe6_tests.log; exit 1; }
tail -n1 gpurun_out/r02_wpe_tests.log; tail -n1 gpurun_out/r02_wpe6_tests.log
for w in 1 6 1 6; do
  CPD_DOWN8_WPE=$w timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --queries 200000 \
     > gpurun_out/r02_wpe$w.json 2> gpurun_out/r02_wpe$w.err || { echo "bench wpe=$w failed"; tail -20 gpurun_out/r02_wpe$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_wpe$w.json'));k=d['kernels'];print('wpe=$w', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')})"
done
for f in 1 2; do
  CPD_FM_WPB=$f timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --queries 200000 \
     > gpurun_out/r02_fmwpb$f.json 2> gpurun_out/r02_fmwpb$f.err || { echo "bench fmwpb=$f failed"; tail -20 gpurun_out/r02_fmwpb$f.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_fmwpb$f.json'));k=d['kernels'];print('fm_wpb=$f', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','first_moves')})"
done
