#!/bin/bash
# Emit overlap A/B: CPD_ASYNC=1 (default) runs each batch's rle_emit on a
# second stream while the next batch's sweeps start; CPD_ASYNC=0 in line.
# CPD_EPRIO=1 puts the emit stream at the lowest priority.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "1 0" "0 0" "1 1" "1 0" "0 0" "1 1"; do
  set -- $cfg
  CPD_ASYNC=$1 CPD_EPRIO=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --queries 200000 \
     > gpurun_out/r02_async$1$2.json 2> gpurun_out/r02_async$1$2.err || { echo "bench $cfg failed"; tail -20 gpurun_out/r02_async$1$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_async$1$2.json'));k=d['kernels'];print('async,eprio=$1$2', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')})"
done
