# two waves per SIMD (2048 resident one-wave groups, 32 lanes each in pass 1) vs the previous build: parity, interleaved A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05al_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05al_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05al_tests.log | head; exit $rc; }
bash tools_scripts/ab_libs.sh r05al ab/libcpd_prev.so 2 || exit 1
out=gpurun_out/r05al_walks.jsonl; : > $out
for lib in A B; do
  if [ $lib = B ]; then export CPD_LIB=$PWD/ab/libcpd_prev.so; else unset CPD_LIB; fi
  timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks >> $out 2>> gpurun_out/r05al.err || exit 1
  echo "$lib walks $(tail -1 $out | cut -c90-160)"
done
