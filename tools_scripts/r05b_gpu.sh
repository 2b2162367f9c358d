mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r05b_tests.log; [ $rc -eq 0 ] || exit $rc
for o in 0 1; do CPD_FM_ORDER=$o timeout -k 10 300 python bench.py --no-cpu --no-search --no-full-build --no-pmc > gpurun_out/r05b_ab_order$o.json 2> gpurun_out/r05b_ab_order$o.err || { tail -5 gpurun_out/r05b_ab_order$o.err; exit 1; }; done
CPD_SEARCH_TRACE=1 timeout -k 10 900 python bench.py > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err; rc=$?; tail -5 gpurun_out/r05b_bench.err; exit $rc
