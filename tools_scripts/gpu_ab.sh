# One GPU call: the GPU parity suite, then the bench with each optimisation
# switched off in turn (CPD_LIVE / CPD_XCD / CPD_SORT, results are identical
# either way) so that one call measures every variant on the same box.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
TAG=${1:-ab}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
echo tests-done
tail -3 $O/gpu_tests_$TAG.log
B="python3 -u $R/bench.py --no-pmc --no-cpu --steps 5"
CPD_TRACE=1 timeout -k 10 300 $B > $O/bench_${TAG}_all.json 2> $O/bench_${TAG}_all.err
echo all-done
for v in LIVE XCD SORT LEAFFM; do
  env CPD_$v=0 timeout -k 10 300 $B > $O/bench_${TAG}_no$v.json 2> $O/bench_${TAG}_no$v.err
  echo no$v-done
done
for f in all noLIVE noXCD noSORT noLEAFFM; do
  python3 - $O/bench_${TAG}_$f.json $f <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["ms"] / 5, 2) for n, v in d["kernels"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], d["queries_per_s"], k)
EOF
done
