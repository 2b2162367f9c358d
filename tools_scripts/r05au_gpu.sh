# fused emit with 8-tile chunks (88 VGPRs, 5 waves/SIMD) vs 16: parity of the variant, interleaved step A/B
mkdir -p gpurun_out
CPD_LIB=$PWD/ab/libcpd_emit8.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05au_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05au_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05au_tests.log | head; exit $rc; }
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for r in 1 2 3; do for lib in A B; do
  if [ $lib = B ]; then export CPD_LIB=$PWD/ab/libcpd_emit8.so; else unset CPD_LIB; fi
  timeout -k 10 300 $B > gpurun_out/r05au_one.json 2> gpurun_out/r05au.err || { tail -5 gpurun_out/r05au.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05au_one.json')); k=p['kernels'].get('rle_emit',{}); print('$lib rep$r', p['value'], p['ms_per_step'], round(k.get('ms',0)/p['steps'],2))" | tee -a gpurun_out/r05au_summary.txt
done; done
