#!/bin/bash
# Bench lines for every workload + the kernel-trace profile of the default one.
set -o pipefail
mkdir -p gpurun_out/prof_r02
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py "$@" > gpurun_out/r02_bench_$name.json 2> gpurun_out/r02_bench_$name.err \
    || { echo "bench $name failed"; tail -20 gpurun_out/r02_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_bench_$name.json'));print('$name', d['value'], d['gteps'], d['queries_per_s'], d['roofline']['kernel'], d['roofline']['frac'], d['query_roofline']['frac'])"
}
run synth1m 420 --steps 20 --warmup 5
run synth4m 600 --workload synth4m --steps 5 --warmup 1
run synth1m_spec 420 --workload synth1m-spec --steps 10 --warmup 2 --no-cpu-partitioned
run melb300k 420 --workload melb300k --steps 10 --warmup 2 --no-cpu-partitioned
cd gpurun_out/prof_r02 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d . -o r02 --output-format csv -- \
    python ../../bench.py --steps 5 --warmup 1 --no-pmc --no-cpu > bench_under_rocprof.json 2> rocprof.err \
    || { echo "rocprof failed"; tail -20 rocprof.err; exit 1; }
ls -R . | head -20
