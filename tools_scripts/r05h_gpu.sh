# deferred emit: parity (rows, drivers' make_cpd_auto pipeline, 1M batch), bench A/B, trace;
# search: adaptive growth (parity, fscale-0 leg)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py tests/test_gpu_scale_1m.py tests/test_gpu_index_stream.py tests/test_gpu_search.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r05h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05h_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05h_tests.log | head; exit $rc; }
for d in 1 0; do CPD_EMIT_DEFER=$d timeout -k 10 400 python bench.py --no-cpu --no-search --no-full-build > gpurun_out/r05h_defer$d.json 2> gpurun_out/r05h_defer$d.err || { tail -5 gpurun_out/r05h_defer$d.err; exit 1; }; done
out=gpurun_out/r05h_search_ab.jsonl; : > $out
for gr in 0 4; do CPD_SEARCH_GROW=$gr CPD_SEARCH_TRACE=1 timeout -k 10 300 python tools_scripts/search_ab.py --fscale 0 >> $out 2>> gpurun_out/r05h_search_ab.err || { tail -5 gpurun_out/r05h_search_ab.err; exit 1; }; done
bash tools_scripts/trace_ab.sh r05h CPD_EMIT_DEFER "1"
