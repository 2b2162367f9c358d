#!/bin/bash
# Round 3, call l: in-kernel multi-level launches for the narrow top levels
# (sweep_up_tail, sweep_down8_head): parity under default and switches, then
# bench A/B against one launch per level.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03l_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03l_tests.log; exit 1; }
tail -2 gpurun_out/r03l_tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 200000 \
      > gpurun_out/r03l_$tag.json 2> gpurun_out/r03l_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r03l_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03l_$tag.json'));k=d['kernels'];print('$tag', d['value'], d['ms_per_step'], {n:round(v['ms']/10,2) for n,v in k.items() if n in ('sweep_down','sweep_up','first_moves','rle_count','rle_emit')}, d['roofline']['frac'], d['parity_sample_bit_exact'])"
}
for rep in 1 2; do
  run tail_$rep CPD_TAIL_UP=64 || exit 1
  run notail_$rep CPD_TAIL_UP=0 CPD_TAIL_DN=0 || exit 1
  run upbig_$rep CPD_TAIL_UP=256 CPD_TAIL_DN=256 || exit 1
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/trace_r03l --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 4 --queries 1000 > $GRAFT_REPO_ROOT/gpurun_out/trace_r03l.json 2> $GRAFT_REPO_ROOT/gpurun_out/trace_r03l.err \
    || { echo "trace failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/trace_r03l.err; exit 1; }
echo trace-done
