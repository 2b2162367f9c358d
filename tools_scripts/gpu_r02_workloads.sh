#!/bin/bash
# Full -m gpu suite, then the default bench line and the other workloads.
set -o pipefail
TAG=${1:-r02f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=10 \
    > gpurun_out/${TAG}_gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('default', d['value'], d['config']['rows_per_step_per_gpu'], d['roofline']['frac'], d['queries_per_s'], d['parity_sample_bit_exact'])"
for w in melb300k synth4m synth1m-spec; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu --steps 10 > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err \
      || { echo "bench $w failed"; tail -20 gpurun_out/${TAG}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$w.json'));print('$w', d['value'], d['config']['rows_per_step_per_gpu'], d['roofline']['frac'], d['queries_per_s'], d['parity_sample_bit_exact'])"
done
if [ "$2" = "prof" ]; then
  R=$PWD; cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG --output-format csv \
      -- python3 $R/bench.py --no-pmc --no-cpu > $R/gpurun_out/prof_${TAG}_bench.json 2> $R/gpurun_out/prof_${TAG}_bench.err \
      || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_${TAG}_bench.err; exit 1; }
  echo prof-done
fi
