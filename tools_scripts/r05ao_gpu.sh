# fscale 0 with lanes-per-wave: growth adaptive vs 2x vs 4x, and first capacity 2^13 vs 2^14
mkdir -p gpurun_out
out=gpurun_out/r05ao_ab.jsonl; : > $out
for v in "CPD_SEARCH_GROW=0" "CPD_SEARCH_GROW=2" "CPD_SEARCH_GROW=4"; do
  env $v CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 >> $out 2>> gpurun_out/r05ao.err || { tail -5 gpurun_out/r05ao.err; exit 1; }
  echo "$v $(tail -1 $out | cut -c90-180)"
done
for c in 8192 32768; do
  CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 --capacity $c --capacity-max 4194304 --frac 0.85 >> $out 2>> gpurun_out/r05ao.err || { tail -5 gpurun_out/r05ao.err; exit 1; }
  echo "cap $c $(tail -1 $out | cut -c90-180)"
done
