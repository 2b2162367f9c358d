# One GPU call: rocprofv3 kernel trace of a 2-step bench (per-dispatch times
# of every sweep level), summarised by tools_scripts/trace_levels.py.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
TAG=${1:-lv}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$TAG --output-format csv -- python3 $R/bench.py --no-pmc --no-cpu --steps 2 --warmup 1 --queries 100000 > $O/trace_${TAG}_bench.json 2> $O/trace_${TAG}_bench.err
echo trace-done
python3 $R/tools_scripts/trace_levels.py $O/trace_$TAG > $O/trace_${TAG}_levels.txt
head -80 $O/trace_${TAG}_levels.txt
