# fused RLE emit: parity + switches, bench A/B fused / unfused; then the
# fscale-0 search: lanes in flight (CPD_SEARCH_WAVES) x first-pass capacity
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py tests/test_gpu_scale_1m.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05d_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05d_tests.log | head; exit $rc; }
for f in 1 0; do CPD_RLE_FUSED=$f timeout -k 10 400 python bench.py --no-cpu --no-search --no-full-build > gpurun_out/r05d_fused$f.json 2> gpurun_out/r05d_fused$f.err || { tail -5 gpurun_out/r05d_fused$f.err; exit 1; }; done
out=gpurun_out/r05d_search_ab.jsonl; : > $out
run() { local w=$1; shift; CPD_SEARCH_WAVES=$w CPD_SEARCH_TRACE=1 timeout -k 10 300 python tools_scripts/search_ab.py "$@" >> $out 2>> gpurun_out/r05d_search_ab.err || { tail -5 gpurun_out/r05d_search_ab.err; exit 1; }; }
run 1024
run 512
run 384
run 256
run 384 --capacity 65536 --capacity-max 524288 --frac 0.85
run 256 --capacity 131072 --capacity-max 524288 --frac 0.85
echo done
