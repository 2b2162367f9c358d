# batch cap with packed rows: 24576 vs 28672 (interleaved x2, no PMC)
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for r in 1 2; do for b in 24576 28672; do
  CPD_BATCH_MAX=$b timeout -k 10 300 $B > gpurun_out/r05am_one.json 2> gpurun_out/r05am.err || { tail -5 gpurun_out/r05am.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05am_one.json')); print('cap $b rep$r', p['config']['rows_per_step_per_gpu'], p['value'], p['ms_per_step'])" | tee -a gpurun_out/r05am_summary.txt
done; done
