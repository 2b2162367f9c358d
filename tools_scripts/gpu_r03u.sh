#!/bin/bash
# Round 3, call u: contraction priority weights (CPD_CH_PRIO = edge
# difference, contracted neighbours, depth) against the sweeps: levels, arcs
# and the bench step at each (own plan cache per setting; rows are the same
# under every hierarchy).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for pr in ${PRIOS:-8,2,3 8,2,6 8,2,12 4,2,3}; do
  tag=$(echo $pr | tr , _)
  CPD_CH_PRIO=$pr CPD_BENCH_CACHE=/tmp/cpd-prio-$tag timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 200000 \
      > gpurun_out/r03u_$tag.json 2> gpurun_out/r03u_$tag.err || { echo "bench $pr failed"; tail -20 gpurun_out/r03u_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03u_$tag.json'));k=d['kernels'];print('$pr', d['value'], d['ms_per_step'], d['hierarchy']['arcs'], d['hierarchy']['levels'], d['hierarchy']['build_s'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves')}, d['roofline']['frac'])"
done
