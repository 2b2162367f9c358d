#!/bin/bash
# Bench A/B over one environment switch, with a step timeline per value.
#   tools_scripts/gpu_ab_env_trace.sh TAG VAR "v1 v2 ..." [batch]
set -o pipefail
TAG=$1; VAR=$2; VALUES=$3; B=${4:-28672}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VALUES; do
  env $VAR=$v timeout -k 10 400 python bench.py --steps 20 --warmup 2 --batch $B --no-cpu --no-pmc \
      --no-search --no-full-build --queries 100000 > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err \
      || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$v.json'));k=d['kernels'];print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sample_bit_exact'), {n:(x['launches'], round(x['ms']/max(1,x['launches']),3), x['GBps']) for n,x in k.items()})"
  env $VAR=$v bash tools_scripts/trace_steps.sh ${TAG}_$v "$B" | tail -16 || exit 1
done
