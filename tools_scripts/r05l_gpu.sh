# up-sweep head before the first moves (CPD_UP_HEAD): parity, bench A/B over the head length, traces
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_drivers.py tests/test_gpu_index_stream.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05l_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05l_tests.log | head; exit $rc; }
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for h in -1 0 8 24 64; do CPD_UP_HEAD=$h timeout -k 10 300 $B > gpurun_out/r05l_h$h.json 2> gpurun_out/r05l_h$h.err || { tail -5 gpurun_out/r05l_h$h.err; exit 1; }; echo "h$h $(cut -c90-200 gpurun_out/r05l_h$h.json)"; done

bash tools_scripts/trace_ab.sh r05l CPD_UP_HEAD "0 24"
