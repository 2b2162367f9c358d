# fscale-0 first-pass capacity with resumable passes (explicit capacity, auto share and growth)
mkdir -p gpurun_out
out=gpurun_out/r05y_cap_ab.jsonl; : > $out
for c in 4096 8192 16384 32768; do
  CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 --capacity $c --capacity-max 4194304 --frac 0.85 >> $out 2>> gpurun_out/r05y_cap_ab.err || { tail -5 gpurun_out/r05y_cap_ab.err; exit 1; }
  echo "cap $c $(tail -1 $out | cut -c1-200)"
done
