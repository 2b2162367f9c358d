#!/bin/bash
# Query kernel knob sweep (one process per setting: the knobs are read once).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r02_qsweep.jsonl
: > $O
run() { env "$@" timeout -k 10 120 python tools_scripts/query_ab.py >> $O || { echo "failed: $*"; exit 1; }; tail -1 $O; }
run CPD_TS_V1=1
for ilp in 1 2; do for wv in 8192 4096 2048 1024 512; do run CPD_TS_ILP=$ilp CPD_TS_WAVES=$wv; done; done
timeout -k 10 60 rocprofv3 -L > gpurun_out/r02_counters.txt 2>&1 || true
