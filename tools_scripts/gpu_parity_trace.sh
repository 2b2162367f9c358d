#!/bin/bash
# The build's parity subset (parity, 1M at size, switches), then step
# timelines per batch width and one plain bench line (no profiler).
#   tools_scripts/gpu_parity_trace.sh TAG "28672 24576" [tests...]
set -o pipefail
TAG=$1; BATCHES=${2:-28672}; shift 2
TESTS=${*:-tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_switches.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -50 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
bash tools_scripts/trace_steps.sh $TAG "$BATCHES" || exit 1
for b in $BATCHES; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 2 --batch $b --no-cpu --no-pmc --no-search \
      --no-full-build --queries 100000 > gpurun_out/${TAG}_bench_b$b.json 2> gpurun_out/${TAG}_bench_b$b.err \
      || { echo "bench $b failed"; tail -20 gpurun_out/${TAG}_bench_b$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_b$b.json'));k=d['kernels'];print('bench b=$b', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sample_bit_exact'), {n:(x['launches'], round(x['ms']/max(1,x['launches']),3), x['GBps']) for n,x in k.items()})"
done
