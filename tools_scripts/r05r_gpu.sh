# pass-1 order by heuristic (CPD_SEARCH_ORDER): search parity, fscale 0 / 0.1 A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05r_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05r_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05r_tests.log | head; exit $rc; }
out=gpurun_out/r05r_search_ab.jsonl; : > $out
for o in 1 0; do
  for fs in 0 0.1; do CPD_SEARCH_ORDER=$o CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale $fs >> $out 2>> gpurun_out/r05r_search_ab.err || { tail -5 gpurun_out/r05r_search_ab.err; exit 1; }; tail -1 $out | cut -c1-220; done
done
