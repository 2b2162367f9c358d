# walks-form queued waves default: search + driver parity tests, then the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_drivers.py tests/test_gpu_switches.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ba_test.log 2>&1 || { tail -40 gpurun_out/r05ba_test.log; exit 1; }
tail -2 gpurun_out/r05ba_test.log
timeout -k 10 700 python bench.py > gpurun_out/r05ba_bench.json 2> gpurun_out/r05ba_bench.err || { tail -20 gpurun_out/r05ba_bench.err; exit 1; }
python - <<'PY'
import json
b = json.load(open("gpurun_out/r05ba_bench.json"))
cs = b["cpd_search"]
print("rows/s", b["value"], "walks", cs["walks_form"]["queries_per_s"], "tables", cs["queries_per_s"], "fs0", cs["fscale0"]["queries_per_s"],
      "fifo cpd", b["full_build"]["serve"]["cpd_search"]["queries_per_s"], b["full_build"]["serve"]["cpd_search"]["bit_exact"])
PY
