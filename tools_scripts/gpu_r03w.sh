#!/bin/bash
# Round 3, call w: the other workloads' bench lines on the final tree
# (synth1m-spec, melb300k stand-in, synth4m = configs[4] worker 0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in synth1m-spec melb300k synth4m; do
  timeout -k 10 500 python bench.py --workload $wl --no-cpu --no-full-build > gpurun_out/r03w_$wl.json 2> gpurun_out/r03w_$wl.err \
      || { echo "bench $wl failed"; tail -20 gpurun_out/r03w_$wl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03w_$wl.json'));print('$wl', d['value'], d['ms_per_step'], d['gteps'], d['queries_per_s'], d.get('queries_per_s_rle'), d['mean_runs_per_row'], d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['frac'], d['hierarchy'], d.get('worker_index_build_s'))"
done
for nw in 256 1024 4096; do
  CPD_UP_NARROW=$nw timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 200000 \
      > gpurun_out/r03w_narrow$nw.json 2> gpurun_out/r03w_narrow$nw.err || { echo "bench narrow $nw failed"; tail -20 gpurun_out/r03w_narrow$nw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03w_narrow$nw.json'));k=d['kernels'];print('narrow=$nw', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')})"
done
for ln in 65536 131072 262144; do
  CPD_CH_LANES=$ln timeout -k 10 200 python tools_scripts/ch_gpu_time.py > gpurun_out/r03w_lanes$ln.log 2>&1 || { echo "timing lanes $ln failed"; exit 1; }
  echo "lanes=$ln"; grep -E "ch-gpu\] [0-9]+ rounds|GPU plan" gpurun_out/r03w_lanes$ln.log | tail -2
done
