# 16-B heap entries (f, column, slot): search parity, A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05w_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05w_tests.log | head; exit $rc; }
out=gpurun_out/r05w_search_ab.jsonl; : > $out
for fs in 0 0.1; do CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale $fs >> $out 2>> gpurun_out/r05w_search_ab.err || { tail -5 gpurun_out/r05w_search_ab.err; exit 1; }; tail -1 $out | cut -c1-220; done
CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks >> $out 2>> gpurun_out/r05w_search_ab.err || { tail -5 gpurun_out/r05w_search_ab.err; exit 1; }; tail -1 $out | cut -c1-220
