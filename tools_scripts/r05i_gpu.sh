# CU reservation for the up-sweep stream: bench A/B (0, 1, 2, 1 emit-only), parity at 2, trace at the best
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for q in 0 1 2 3; do CPD_CU_RESERVE=$q timeout -k 10 300 $B > gpurun_out/r05i_cu$q.json 2> gpurun_out/r05i_cu$q.err || { tail -5 gpurun_out/r05i_cu$q.err; exit 1; }; echo "cu$q $(cut -c1-160 gpurun_out/r05i_cu$q.json)"; done
CPD_CU_RESERVE=1 CPD_CU_RESERVE_MAIN=0 timeout -k 10 300 $B > gpurun_out/r05i_cu1e.json 2> gpurun_out/r05i_cu1e.err || { tail -5 gpurun_out/r05i_cu1e.err; exit 1; }
CPD_CU_RESERVE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_scale_1m.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05i_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools_scripts/trace_ab.sh r05i CPD_CU_RESERVE "1 2"
