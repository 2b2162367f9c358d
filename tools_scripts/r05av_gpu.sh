# fused emit's occupancy capped by extra LDS (CPD_EMIT_LDS): interleaved step A/B
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for r in 1 2; do for x in 0 49152 77824; do
  CPD_EMIT_LDS=$x timeout -k 10 300 $B > gpurun_out/r05av_one.json 2> gpurun_out/r05av.err || { tail -5 gpurun_out/r05av.err; exit 1; }
  python3 -c "
import json; p=json.load(open('gpurun_out/r05av_one.json')); print('lds $x rep$r', p['value'], p['ms_per_step'])" | tee -a gpurun_out/r05av_summary.txt
done; done
