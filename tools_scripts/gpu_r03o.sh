#!/bin/bash
# Round 3, call o: the next batch's up-sweep split around the first moves
# (CPD_UP_SPLIT): parity + switches, then bench A/B and a step trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03o_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03o_tests.log; exit 1; }
tail -2 gpurun_out/r03o_tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 200000 \
      > gpurun_out/r03o_$tag.json 2> gpurun_out/r03o_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r03o_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03o_$tag.json'));k=d['kernels'];print('$tag', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')})"
}
for rep in 1 2; do
  run split_$rep CPD_UP_SPLIT=1 || exit 1
  run nosplit_$rep CPD_UP_SPLIT=0 || exit 1
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace_r03o --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 4 --queries 1000 > $GRAFT_REPO_ROOT/gpurun_out/trace_r03o.json 2> $GRAFT_REPO_ROOT/gpurun_out/trace_r03o.err \
    || { echo "trace failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/trace_r03o.err; exit 1; }
echo trace-done
