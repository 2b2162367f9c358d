# built rows at the packed width: parity (rows, drivers, 1M batch, index stream, switches, search), PMC A/B vs nibble rows
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_switches.py tests/test_gpu_drivers.py tests/test_gpu_index_stream.py tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05af_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05af_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05af_tests.log | head; exit $rc; }
B="python bench.py --no-cpu --no-search --no-full-build"
for v in "CPD_ROWS_NIBBLE=0" "CPD_ROWS_NIBBLE=1"; do
  env $v timeout -k 10 400 $B > gpurun_out/r05af_$v.json 2> gpurun_out/r05af_$v.err || { tail -5 gpurun_out/r05af_$v.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05af_$v.json')); e=p['pmc_traffic_per_launch'].get('rle_emit',{})
print('$v', p['value'], p['ms_per_step'], p['step_pmc']['GB'], round(e.get('read',0)/1e9,2), round(e.get('write',0)/1e9,2), p.get('rows_per_s_runs'))"
done
