# persistent fused emit (CPD_EMIT_PERSIST=w workgroups per CU): parity, interleaved step A/B, trace at the best
mkdir -p gpurun_out
CPD_EMIT_PERSIST=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05aw_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05aw_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05aw_tests.log | head; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_switches.py -x -q -k "EMIT_PERSIST" --timeout 300 --timeout-method thread > gpurun_out/r05aw_sw.log 2>&1; rc=$?; tail -1 gpurun_out/r05aw_sw.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for r in 1 2; do for w in 0 1 2 3; do
  CPD_EMIT_PERSIST=$w timeout -k 10 300 $B > gpurun_out/r05aw_one.json 2> gpurun_out/r05aw.err || { tail -5 gpurun_out/r05aw.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05aw_one.json')); print('persist $w rep$r', p['value'], p['ms_per_step'])" | tee -a gpurun_out/r05aw_summary.txt
done; done
