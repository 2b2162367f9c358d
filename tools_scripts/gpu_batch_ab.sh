#!/bin/bash
# Bench A/B over the batch size (rows per step) on the default workload.
set -o pipefail
mkdir -p gpurun_out
for b in ${BATCHES:-16384 20480 24576}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search \
      --queries 100000 --batch $b > gpurun_out/batch_b$b.json 2> gpurun_out/batch_b$b.err \
      || { echo "bench batch $b failed"; tail -5 gpurun_out/batch_b$b.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/batch_b$b.json'));k=d['kernels'];print('batch=$b', d['value'], d['ms_per_step'], {n:round(x['ms']/x['launches'],3) for n,x in k.items()})"
done
