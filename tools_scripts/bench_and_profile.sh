# One GPU call: the default bench line (with its PMC child passes and CPU
# baseline), then a rocprofv3 kernel-trace of the same workload for profiles/.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
timeout -k 10 600 python3 -u $R/bench.py > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err
echo bench-done
cat $R/gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG --output-format csv -- python3 $R/bench.py --no-pmc --no-cpu > $R/gpurun_out/prof_${TAG}_bench.json 2> $R/gpurun_out/prof_${TAG}_bench.err
echo prof-done
