# walks form with one walk call site in the room check: parity, interleaved A/B vs the previous build
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05as_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05as_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05as_tests.log | head; exit $rc; }
out=gpurun_out/r05as_walks.jsonl; : > $out
for r in 1 2; do for lib in A B; do
  if [ $lib = B ]; then export CPD_LIB=$PWD/ab/libcpd_prev.so; else unset CPD_LIB; fi
  for fs in 0.1 0; do
  timeout -k 10 200 python tools_scripts/search_ab.py --fscale $fs --tables walks --queries 16384 > gpurun_out/r05as_one.json 2>> gpurun_out/r05as.err || { tail -5 gpurun_out/r05as.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05as_one.json')); d['lib']='$lib'; print(json.dumps(d))" >> $out
  echo "$lib rep$r fs $fs walks $(python3 -c "import json; print(json.load(open('gpurun_out/r05as_one.json'))['qps'])")"
  done
done; done
