# One GPU call: bench (no PMC / CPU leg) under each workgroup-size switch.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for cfg in ${CFGS:-"X=0" "CPD_DOWN8_WPB=1" "CPD_DOWN8_WPB=4" "CPD_FM_WPB=1" "CPD_FM_WPB=4"}; do
  env $cfg timeout -k 10 300 python3 -u $R/bench.py --no-pmc --no-cpu --steps 5 > $O/bench_wpb.json 2> $O/bench_wpb.err
  python3 - $O/bench_wpb.json "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["ms"] / d["steps"], 2) for n, v in d["kernels"].items()}
print(sys.argv[2], d["value"], k["sweep_down"], k["first_moves"])
PY
done
