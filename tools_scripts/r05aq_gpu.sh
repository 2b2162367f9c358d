# run-word decode with the next tile prefetched: parity (rows, drivers incl. --format rle, 1M batch, index stream), decode time
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py tests/test_gpu_scale_1m.py tests/test_gpu_index_stream.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05aq_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05aq_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r05aq_tests.log | head; exit $rc; }
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000 > gpurun_out/r05aq_one.json 2> gpurun_out/r05aq.err || { tail -5 gpurun_out/r05aq.err; exit 1; }
python3 -c "
import json; p=json.load(open('gpurun_out/r05aq_one.json')); print(p['value'], p['ms_per_step'], p.get('runs_form'))" | tee -a gpurun_out/r05aq_summary.txt
done
