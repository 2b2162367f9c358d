#!/bin/bash
# Per-level down-sweep: kernel trace + FETCH/WRITE passes of one build step.
set -o pipefail
mkdir -p gpurun_out/lv
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-pmc --no-cpu --queries 1000 > /dev/null 2> gpurun_out/lv/plan.err || exit 1
cd gpurun_out/lv
timeout -k 10 300 rocprofv3 --kernel-trace -d tr --output-format csv -- python $R/bench.py --pmc-child --steps 1 --warmup 0 > tr.log 2>&1 || { tail tr.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d fe --output-format csv -- python $R/bench.py --pmc-child --steps 1 --warmup 0 > fe.log 2>&1 || { tail fe.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d wr --output-format csv -- python $R/bench.py --pmc-child --steps 1 --warmup 0 > wr.log 2>&1 || { tail wr.log; exit 1; }
python $R/tools_scripts/level_pmc.py tr fe wr ../${1:-r02_down_levels_pmc.txt}
rm -rf tr fe wr
