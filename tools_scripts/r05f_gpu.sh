# search kernel: prefetched pops + batched pushes — parity, then the legs
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05f_tests.log | head; exit $rc; }
out=gpurun_out/r05f_search_ab.jsonl; : > $out
run() { CPD_SEARCH_TRACE=1 timeout -k 10 300 python tools_scripts/search_ab.py "$@" >> $out 2>> gpurun_out/r05f_search_ab.err || { tail -5 gpurun_out/r05f_search_ab.err; exit 1; }; }
run --fscale 0
run --fscale 0.1
run --fscale 0.1 --tables walks
echo done
