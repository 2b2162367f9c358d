# first-moves workgroup shape (CPD_FM_WPB) x up-sweep head (CPD_UP_HEAD): bench A/B, traces
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for w in 4 2; do for h in -1 0 24; do CPD_FM_WPB=$w CPD_UP_HEAD=$h timeout -k 10 300 $B > gpurun_out/r05m_w${w}h$h.json 2> gpurun_out/r05m_w${w}h$h.err || { tail -5 gpurun_out/r05m_w${w}h$h.err; exit 1; }; echo "w$w h$h $(cut -c90-200 gpurun_out/r05m_w${w}h$h.json)"; done; done
CPD_FM_WPB=4 bash tools_scripts/trace_ab.sh r05m CPD_UP_HEAD "24 -1"
