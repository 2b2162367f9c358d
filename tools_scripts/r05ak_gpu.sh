# lanes per wave = the fewest (multiple of 8) that keep one wave per SIMD: parity, fscale 0 / 0.1 / walks
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05ak_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05ak_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05ak_tests.log | head; exit $rc; }
out=gpurun_out/r05ak_search_ab.jsonl; : > $out
for r in 1 2; do
  for fs in 0 0.1; do CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale $fs >> $out 2>> gpurun_out/r05ak.err || { tail -5 gpurun_out/r05ak.err; exit 1; }; echo "fs $fs $(tail -1 $out | cut -c90-200)"; done
done
CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks >> $out 2>> gpurun_out/r05ak.err || { tail -5 gpurun_out/r05ak.err; exit 1; }; echo "walks $(tail -1 $out | cut -c90-200)"
