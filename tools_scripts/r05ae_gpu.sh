# wide (16-B) packed-table stores in the fused emit: parity, PMC A/B (wide / per-lane / 4-bit tables), then the other workloads' lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_switches.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05ae_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05ae_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05ae_tests.log | head; exit $rc; }
B="python bench.py --no-cpu --no-search --no-full-build"
for v in "CPD_EMIT_WIDE=1" "CPD_EMIT_WIDE=0" "CPD_TABLE_BITS=4"; do
  env $v timeout -k 10 400 $B > gpurun_out/r05ae_$v.json 2> gpurun_out/r05ae_$v.err || { tail -5 gpurun_out/r05ae_$v.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05ae_$v.json')); e=p['pmc_traffic_per_launch'].get('rle_emit',{})
print('$v', p['value'], p['ms_per_step'], p['step_pmc']['GB'], round(e.get('read',0)/1e9,2), round(e.get('write',0)/1e9,2))"
done
