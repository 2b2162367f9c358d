# packed vs nibble built rows, interleaved x3 (no PMC), plus emit wide/narrow stores on packed rows
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for r in 1 2 3; do for v in "CPD_ROWS_NIBBLE=0" "CPD_ROWS_NIBBLE=1" "CPD_EMIT_WIDE=0"; do
  env $v timeout -k 10 300 $B > gpurun_out/r05ag_one.json 2> gpurun_out/r05ag.err || { tail -5 gpurun_out/r05ag.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05ag_one.json')); print('$v rep$r', p['value'], p['ms_per_step'], p.get('rows_per_s_runs'))" | tee -a gpurun_out/r05ag_summary.txt
done; done
