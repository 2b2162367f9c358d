# one begin() call site in the search kernel: parity, interleaved A/B (tables fscale 0 / 0.1, walks 0.1) vs the previous build
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05at_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05at_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05at_tests.log | head; exit $rc; }
bash tools_scripts/ab_libs.sh r05at ab/libcpd_prev.so 2 || exit 1
for r in 1 2; do for lib in A B; do
  if [ $lib = B ]; then export CPD_LIB=$PWD/ab/libcpd_prev.so; else unset CPD_LIB; fi
  timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks > gpurun_out/r05at_one.json 2>> gpurun_out/r05at.err || exit 1
  echo "$lib rep$r walks $(python3 -c "import json; print(json.load(open('gpurun_out/r05at_one.json'))['qps'])")"
done; done
