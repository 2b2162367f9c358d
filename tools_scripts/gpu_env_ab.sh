#!/bin/bash
# GPU parity subset, then a bench A/B over one environment switch.
#   tools_scripts/gpu_env_ab.sh TAG VAR "v1 v2 ..." [tests...]
# (default tests: the parity suite + the 1M at-size tests; "none" skips them)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; VAR=$2; VALUES=$3; shift 3
TESTS=${*:-tests/test_gpu_parity.py tests/test_gpu_scale_1m.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search \
      --queries 100000 ${BENCH_ARGS} > gpurun_out/${TAG}_b$v.json 2> gpurun_out/${TAG}_b$v.err \
      || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_b$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_b$v.json'));k=d['kernels'];print('$VAR=$v', d['value'], d['ms_per_step'], d.get('parity_sample_bit_exact'), {n:(round(x['ms']/x['launches'],3), round(x['GBps'])) for n,x in k.items()})"
done
