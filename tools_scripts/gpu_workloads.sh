#!/bin/bash
# The bench's other workloads on the current tree, one default line each.
#   tools_scripts/gpu_workloads.sh TAG "synth1m-spec melb300k synth4m"
set -o pipefail
TAG=$1; WLS=${2:-"synth1m-spec melb300k synth4m"}
mkdir -p gpurun_out
for w in $WLS; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err \
    || { echo "$w failed"; tail -20 gpurun_out/${TAG}_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('gteps'), d.get('queries_per_s'), d['config'].get('rows_per_step_per_gpu'), d.get('parity_sample_bit_exact'))"
done
