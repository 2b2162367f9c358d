# walks form at fscale 0 (long searches): resident 1024 vs the new walks default 2048
mkdir -p gpurun_out
out=gpurun_out/r05az_ab.jsonl; : > $out
for r in 1 2; do for v in 1024 2048; do
  CPD_SEARCH_RESIDENT=$v CPD_SEARCH_TRACE=1 timeout -k 10 300 python tools_scripts/search_ab.py --fscale 0 --tables walks --queries 16384 >> $out 2>> gpurun_out/r05az.err || { tail -5 gpurun_out/r05az.err; exit 1; }
  echo "walks fs0 resident $v $(tail -1 $out | grep -o '"qps": [0-9.]*')"
done; done
for r in 1 2; do
  timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks >> $out 2>> gpurun_out/r05az.err && echo "walks fs0.1 default $(tail -1 $out | grep -o '"qps": [0-9.]*')"
done
