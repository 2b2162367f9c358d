# walks form (fscale 0.1): first capacity 8192 (policy) vs 16384 vs 32768
mkdir -p gpurun_out
out=gpurun_out/r05ap_ab.jsonl; : > $out
for r in 1 2; do
CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks >> $out 2>> gpurun_out/r05ap.err || { tail -5 gpurun_out/r05ap.err; exit 1; }
echo "policy $(tail -1 $out | cut -c90-180)"
for c in 16384 32768; do
  CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 --tables walks --capacity $c --capacity-max 4194304 --frac 0.85 >> $out 2>> gpurun_out/r05ap.err || { tail -5 gpurun_out/r05ap.err; exit 1; }
  echo "cap $c $(tail -1 $out | cut -c90-180)"
done; done
