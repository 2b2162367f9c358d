# query-file reader (reused buffers, one-scan lines): drivers parity + the serve leg
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_drivers.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05ab_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05ab_tests.log | head; exit $rc; }
timeout -k 10 600 python bench.py --full-build-only --no-cpu > gpurun_out/r05ab_fb.json 2> gpurun_out/r05ab_fb.err || { tail -5 gpurun_out/r05ab_fb.err; exit 1; }
python3 -c "
import json; p=json.load(open('gpurun_out/r05ab_fb.json')); sv=(p.get('full_build') or {}).get('serve') or {}
print(json.dumps({k: sv.get(k) for k in ('ready_s','bit_exact')}), json.dumps(sv.get('table_search'))[:600])"
