# fewer lanes per wave in late passes (CPD_SEARCH_LPW_MIN): parity at 8, fscale-0 A/B
mkdir -p gpurun_out
CPD_SEARCH_LPW_MIN=8 timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05aj_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05aj_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05aj_tests.log | head; exit $rc; }
out=gpurun_out/r05aj_lpw_ab.jsonl; : > $out
for r in 1 2; do for l in 64 32 16 8; do
  CPD_SEARCH_LPW_MIN=$l CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 >> $out 2>> gpurun_out/r05aj.err || { tail -5 gpurun_out/r05aj.err; exit 1; }
  echo "lpw_min $l $(tail -1 $out | cut -c90-200)"
done; done
