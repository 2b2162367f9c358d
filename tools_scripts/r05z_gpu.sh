# fscale 0: lanes (CPD_SEARCH_WAVES: queries refill a wave's lanes) x first capacity
mkdir -p gpurun_out
out=gpurun_out/r05z_waves_ab.jsonl; : > $out
for w in 512 256 128; do for c in 16384 4096; do
  CPD_SEARCH_WAVES=$w CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 --capacity $c --capacity-max 4194304 --frac 0.85 >> $out 2>> gpurun_out/r05z_waves_ab.err || { tail -5 gpurun_out/r05z_waves_ab.err; exit 1; }
  echo "waves $w cap $c $(tail -1 $out | cut -c100-200)"
done; done
