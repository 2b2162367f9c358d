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
