# fscale 0: growth steps (adaptive 2-4x vs 2x) with the 2^14 first pass; twice each
mkdir -p gpurun_out
out=gpurun_out/r05aa_grow_ab.jsonl; : > $out
for r in 1 2; do for gr in 0 2; do
  CPD_SEARCH_GROW=$gr CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 >> $out 2>> gpurun_out/r05aa_grow_ab.err || { tail -5 gpurun_out/r05aa_grow_ab.err; exit 1; }
  echo "grow $gr $(tail -1 $out | cut -c90-200)"
done; done
