#!/bin/bash
# Round 3: CU partition for the early up-sweep (CPD_UP_CUS) A/B, parity of the
# partitioned path, and a kernel trace at the chosen setting.
set -o pipefail
TAG=${1:-r03g}
CUS=${2:-16}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
CPD_UP_CUS=$CUS timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "hint or multi_slab or rows_bit_exact" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
B="python bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 10"
for c in 0 8 16 32; do
  CPD_UP_CUS=$c timeout -k 10 400 $B > gpurun_out/${TAG}_cus$c.json 2> gpurun_out/${TAG}_cus$c.err || { echo "bench cus$c failed"; tail -5 gpurun_out/${TAG}_cus$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_cus$c.json'));print('cus$c', d['value'], d['ms_per_step'], {k:round(v['ms']/d['steps'],2) for k,v in d['kernels'].items()})"
done
cd /tmp
CPD_UP_CUS=$CUS timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_$TAG --output-format csv \
    -- python3 $R/bench.py --no-cpu --no-full-build --no-search --no-pmc --steps 4 --queries 1000 > $R/gpurun_out/trace_${TAG}.json 2> $R/gpurun_out/trace_${TAG}.err \
    || { echo "trace failed"; tail -5 $R/gpurun_out/trace_${TAG}.err; exit 1; }
echo trace-done
