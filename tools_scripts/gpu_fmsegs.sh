# One GPU call: GPU parity suite (default CPD_FM_SEGS=2), then the bench with
# PMC passes at CPD_FM_SEGS=2 and =1 (first-moves write traffic A/B).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_fmsegs.log 2>&1
echo "tests: $(tail -1 $O/gpu_tests_fmsegs.log)"
for v in 2 1; do
  CPD_FM_SEGS=$v timeout -k 10 500 python3 -u $R/bench.py --no-cpu > $O/bench_fmsegs$v.json 2> $O/bench_fmsegs$v.err
  python3 - $O/bench_fmsegs$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["ms"] / d["steps"], 2) for n, v in d["kernels"].items()}
fm = d.get("pmc_traffic_per_launch", {}).get("first_moves", {})
print("segs", sys.argv[2], d["value"], d["ms_per_step"], k, "fm pmc", fm)
PY
done
