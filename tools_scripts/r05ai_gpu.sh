# walks-form search: non-inlined cpd_walk (A, tree) vs inlined (B, previous build), interleaved
mkdir -p gpurun_out
out=gpurun_out/r05ai_walks_ab.jsonl; : > $out
for r in 1 2; do for lib in A B; do
  if [ $lib = B ]; then export CPD_LIB=$PWD/ab/libcpd_prev.so; else unset CPD_LIB; fi
  timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks > gpurun_out/r05ai_one.json 2>> gpurun_out/r05ai.err || { tail -5 gpurun_out/r05ai.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05ai_one.json')); d['lib']='$lib'; print(json.dumps(d))" >> $out
  echo "$lib rep$r walks $(python3 -c "import json; print(json.load(open('gpurun_out/r05ai_one.json'))['qps'])")"
done; done
unset CPD_LIB
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r05ai_tests.log 2>&1; tail -1 gpurun_out/r05ai_tests.log
