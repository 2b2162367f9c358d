# 28672-row default batch: HBM-reserve and 1M-batch parity, drivers, then the default bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hbm_reserve.py tests/test_gpu_scale_1m.py tests/test_gpu_drivers.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05an_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05an_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05an_tests.log | head; exit $rc; }
timeout -k 10 700 python bench.py > gpurun_out/r05an_bench.json 2> gpurun_out/r05an_bench.err || { tail -20 gpurun_out/r05an_bench.err; exit 1; }
cut -c1-400 gpurun_out/r05an_bench.json
