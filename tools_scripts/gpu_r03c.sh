#!/bin/bash
# Round 3, call c: does the early up-sweep overlap?  Step time with the
# default queues, with 8 HW queues, with the overlap off; a kernel trace of
# a short run for the overlap analysis (tools_scripts/overlap_trace.py).
set -o pipefail
TAG=${1:-r03c}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
B="python bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 10"
timeout -k 10 400 $B > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_default.err; exit 1; }
CPD_UP_PRIO=0 timeout -k 10 400 $B > gpurun_out/${TAG}_q8.json 2> gpurun_out/${TAG}_q8.err || { echo "bench noprio failed"; tail -5 gpurun_out/${TAG}_q8.err; exit 1; }
CPD_OVERLAP=0 timeout -k 10 400 $B > gpurun_out/${TAG}_nooverlap.json 2> gpurun_out/${TAG}_nooverlap.err || { echo "bench nooverlap failed"; exit 1; }
for f in default q8 nooverlap; do python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$f.json'));print('$f', d['value'], d['ms_per_step'], {k:round(v['ms']/d['steps'],2) for k,v in d['kernels'].items()})"; done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_$TAG --output-format csv \
    -- python3 $R/bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 4 --queries 1000 > $R/gpurun_out/trace_${TAG}.json 2> $R/gpurun_out/trace_${TAG}.err \
    || { echo "trace failed"; tail -5 $R/gpurun_out/trace_${TAG}.err; exit 1; }
echo trace-done
