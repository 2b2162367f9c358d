#!/bin/bash
# Round 3, call m: A/B of the down head alone / small up tails against one
# launch per level.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 200000 \
      > gpurun_out/r03m_$tag.json 2> gpurun_out/r03m_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r03m_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03m_$tag.json'));k=d['kernels'];print('$tag', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')})"
}
for rep in 1 2; do
  run notail_$rep CPD_TAIL_UP=0 CPD_TAIL_DN=0 || exit 1
  run head64_$rep CPD_TAIL_UP=0 CPD_TAIL_DN=64 || exit 1
  run head256_$rep CPD_TAIL_UP=0 CPD_TAIL_DN=256 || exit 1
  run head64up16_$rep CPD_TAIL_UP=16 CPD_TAIL_DN=64 || exit 1
done
