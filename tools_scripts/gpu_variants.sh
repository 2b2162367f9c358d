# One GPU call: for each prebuilt libcpd variant under variants/ (names given
# as arguments), swap it in, run the GPU parity suite and one bench line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
LIB=$R/distributed-oracle-search_amd/libcpd.so
cp $LIB $O/../variants/.orig.so
for v in "$@"; do
  cp $R/variants/libcpd_$v.so $LIB
  timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$v.log 2>&1
  echo "$v tests: $(tail -1 $O/gpu_tests_$v.log)"
  timeout -k 10 300 python3 -u $R/bench.py --no-pmc --no-cpu --steps 5 > $O/bench_$v.json 2> $O/bench_$v.err
  python3 - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["ms"] / d["steps"], 2) for n, v in d["kernels"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], d["queries_per_s"], k)
PY
done
cp $R/variants/.orig.so $LIB
