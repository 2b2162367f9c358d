# One GPU call: the GPU parity suite (unless SKIP_TESTS=1), then one short
# bench per variant; a variant is a space-free list of VAR=VALUE joined by ','
# ("base" = defaults).  Results are identical in every variant; only speed
# differs.   bash tools_scripts/gpu_knobs.sh TAG base CPD_DSORT=0 CPD_FM_G=4,CPD_FM_WPB=2
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
TAG=$1
shift
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
  echo tests-done
  tail -2 $O/gpu_tests_$TAG.log
fi
B="python3 -u $R/bench.py --no-pmc --no-cpu --steps 5"
for v in "$@"; do
  envs=$(echo "$v" | tr ',' ' ')
  [ "$v" = base ] && envs=""
  env $envs timeout -k 10 300 $B > $O/knob_${TAG}_$v.json 2> $O/knob_${TAG}_$v.err
  python3 - $O/knob_${TAG}_$v.json $v <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["ms"] / 5, 2) for n, v in d["kernels"].items() if v["ms"] / 5 > 0.3}
print(sys.argv[2], d["value"], d["ms_per_step"], k, flush=True)
EOF
done
