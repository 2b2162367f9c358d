# One GPU call: the GPU parity suite, then one bench line without the PMC
# passes and CPU leg, with the per-kernel ms per step printed.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
TAG=${1:-chk}
shift || true
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
echo tests-done
tail -2 $O/gpu_tests_$TAG.log
timeout -k 10 300 python3 -u $R/bench.py --no-pmc --no-cpu --steps 5 "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err
python3 - $O/bench_$TAG.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["ms"] / d["steps"], 2) for n, v in d["kernels"].items()}
print(d["value"], d["ms_per_step"], d["queries_per_s"], d.get("queries_per_s_rle"), d["parity_sample_bit_exact"], k)
PY
