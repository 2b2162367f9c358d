# register-resident fused emit: parity (rows, seams, 1M batch, switches), bench with PMC, trace
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_switches.py tests/test_gpu_drivers.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05j_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05j_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05j_tests.log | head; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu --no-search --no-full-build > gpurun_out/r05j_bench.json 2> gpurun_out/r05j_bench.err || { tail -5 gpurun_out/r05j_bench.err; exit 1; }
cut -c1-200 gpurun_out/r05j_bench.json
bash tools_scripts/trace_ab.sh r05j CPD_EMIT_DEFER "0 1"
