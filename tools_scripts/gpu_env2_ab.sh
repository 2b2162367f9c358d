#!/bin/bash
# Bench A/B over combinations of environment settings, alternating, same box.
#   tools_scripts/gpu_env2_ab.sh TAG "A=1,B=0" "A=0,B=1" ... (extra bench args in BENCH_ARGS)
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu --no-pmc --no-search \
      --no-full-build --queries 100000 ${BENCH_ARGS} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err \
      || { echo "bench $cfg failed"; tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$i.json'));k=d['kernels'];print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], {n:(round(x['ms']/max(1,x['launches']),3), round(x['GBps'])) for n,x in k.items()})"
done
