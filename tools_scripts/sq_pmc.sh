#!/bin/bash
# SQ counters per kernel of a short build-only bench run (one rocprofv3 --pmc
# pass, 8 SQ slots), summed per kernel name by tools_scripts/sq_pmc_sum.py.
#   tools_scripts/sq_pmc.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/pmc_$TAG --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-pmc --no-search --no-full-build \
    --queries 100000 "$@" > $R/gpurun_out/pmc_${TAG}.json 2> $R/gpurun_out/pmc_${TAG}.err ) \
  || { echo "pmc run failed"; tail -20 gpurun_out/pmc_${TAG}.err; exit 1; }
python3 tools_scripts/sq_pmc_sum.py gpurun_out/pmc_$TAG > gpurun_out/pmc_${TAG}_summary.txt && cat gpurun_out/pmc_${TAG}_summary.txt
