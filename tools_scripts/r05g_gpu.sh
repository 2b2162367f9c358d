bash tools_scripts/r05f_gpu.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_switches.py -x -v --timeout 300 --timeout-method thread -k "TS_SHARE or RLE_FUSED or FM_ORDER" > gpurun_out/r05g_switch.log 2>&1; rc=$?; tail -3 gpurun_out/r05g_switch.log; [ $rc -eq 0 ] || exit $rc
for sh in 0 1; do CPD_TS_SHARE=$sh CPD_SEARCH_TRACE=1 timeout -k 10 300 python tools_scripts/query_ab.py --modes dense > gpurun_out/r05g_share$sh.json 2> gpurun_out/r05g_share$sh.err || { tail -5 gpurun_out/r05g_share$sh.err; exit 1; }; done
bash tools_scripts/trace_ab.sh r05e CPD_RLE_FUSED "1 0"
