#!/bin/bash
# Generic switch A/B on the default bench workload: parity suite under every
# value first, then alternating bench runs.
#   tools_scripts/gpu_ab_env.sh TAG VAR "v1 v2 ..." [tests]
# tests: pytest paths run under each value (default tests/test_gpu_parity.py).
# Output: gpurun_out/<TAG>_<VAR><v>_<rep>.json and one summary line per run.
set -o pipefail
tag=$1; var=$2; vals=$3; tests=${4:-tests/test_gpu_parity.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $vals; do
  env "$var=$v" timeout -k 10 400 python -u -m pytest $tests -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/${tag}_tests_$v.log 2>&1 || { echo "TESTS FAILED $var=$v"; tail -30 gpurun_out/${tag}_tests_$v.log; exit 1; }
  echo "$var=$v: $(tail -n1 gpurun_out/${tag}_tests_$v.log)"
done
for rep in 1 2; do
  for v in $vals; do
    out=gpurun_out/${tag}_${var}${v}_$rep
    env "$var=$v" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 200000 \
        > $out.json 2> $out.err || { echo "bench $var=$v failed"; tail -20 $out.err; exit 1; }
    python -c "import json;d=json.load(open('$out.json'));k=d['kernels'];print('$var=$v', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')}, d['roofline']['frac'])"
  done
done
