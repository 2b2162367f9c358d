# fscale 0.1 (short searches), tables and walks forms: CPD_SEARCH_RESIDENT 1024 / 2048 / 4096
mkdir -p gpurun_out
out=gpurun_out/r05ay_ab.jsonl; : > $out
for r in 1 2 3; do for f in tables walks; do for v in 1024 2048 4096; do
  CPD_SEARCH_RESIDENT=$v timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables $f >> $out 2>> gpurun_out/r05ay.err || { tail -5 gpurun_out/r05ay.err; exit 1; }
  echo "$f resident $v $(tail -1 $out | grep -o '"qps": [0-9.]*')"
done; done; done
