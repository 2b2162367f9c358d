#!/bin/bash
# Kernel traces of short bench runs under several settings of one switch:
#   tools_scripts/trace_ab.sh TAG VAR "v1 v2 ..."
# -> gpurun_out/trace_TAG_VAR<v>/ (rocprofv3 --kernel-trace, csv)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; VAR=$2; VALUES=$3
R=$PWD
mkdir -p gpurun_out
cd /tmp
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_${TAG}_$VAR$v \
      -- python3 $R/bench.py --steps 8 --warmup 2 --no-cpu --no-pmc --no-search --no-full-build --queries 100000 \
      > $R/gpurun_out/trace_${TAG}_$VAR$v.json 2> $R/gpurun_out/trace_${TAG}_$VAR$v.err \
      || { echo "trace $VAR=$v failed"; tail -20 $R/gpurun_out/trace_${TAG}_$VAR$v.err; exit 1; }
  echo "$VAR=$v traced"
done
