# fscale 0 with more (queued) waves of fewer lanes: CPD_SEARCH_RESIDENT 1024 / 2048 / 4096
mkdir -p gpurun_out
out=gpurun_out/r05ax_ab.jsonl; : > $out
for r in 1 2; do for v in 1024 2048 4096; do
  CPD_SEARCH_RESIDENT=$v CPD_SEARCH_TRACE=1 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0 >> $out 2>> gpurun_out/r05ax.err || { tail -5 gpurun_out/r05ax.err; exit 1; }
  echo "resident $v $(tail -1 $out | cut -c90-170)"
done; done
CPD_SEARCH_RESIDENT=2048 timeout -k 10 200 python tools_scripts/search_ab.py --fscale 0.1 >> $out 2>> gpurun_out/r05ax.err && echo "resident 2048 fs0.1 $(tail -1 $out | cut -c90-170)"
