# hscale-1 / fscale-0 integer fast paths: search parity, interleaved A/B vs the previous build; then the workloads' bench lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05ah_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05ah_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05ah_tests.log | head; exit $rc; }
bash tools_scripts/ab_libs.sh r05ah ab/libcpd_prev.so 2 || exit 1
bash tools_scripts/r05ad_gpu.sh
