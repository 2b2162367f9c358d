#!/bin/bash
# Bench A/B of this tree's libcpd.so against another build (CPD_LIB), alternating.
#   tools_scripts/gpu_lib_ab.sh TAG LIB_B [rounds] [tests...]  (tests run on LIB_B first)
set -o pipefail
TAG=$1; LIBB=$2; N=${3:-2}; shift 3
mkdir -p gpurun_out
if [ -n "$*" ]; then
  CPD_LIB=$PWD/$LIBB timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for i in $(seq 1 $N); do
  for side in A B; do
    if [ $side = B ]; then export CPD_LIB=$PWD/$LIBB; else unset CPD_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build \
        --queries 100000 > gpurun_out/${TAG}_${side}_$i.json 2> gpurun_out/${TAG}_${side}_$i.err \
      || { echo "$side $i failed"; tail -20 gpurun_out/${TAG}_${side}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${side}_$i.json'));k=d['kernels'];print('$side $i', d['value'], d['ms_per_step'], d['roofline']['frac'], d['lib_src_sha'], {n:round(x['ms']/max(1,x['launches']),3) for n,x in k.items()})"
  done
done
