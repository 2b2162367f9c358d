# first moves' occupancy cap (CPD_FM_LDS) x up-sweep head (CPD_UP_HEAD): bench A/B, trace
mkdir -p gpurun_out
B="python bench.py --no-cpu --no-search --no-full-build --no-pmc --queries 100000"
for l in 13824 20480 16384; do for h in 0 -1; do CPD_FM_LDS=$l CPD_UP_HEAD=$h timeout -k 10 300 $B > gpurun_out/r05n_l${l}h$h.json 2> gpurun_out/r05n_l${l}h$h.err || { tail -5 gpurun_out/r05n_l${l}h$h.err; exit 1; }; echo "l$l h$h $(cut -c90-200 gpurun_out/r05n_l${l}h$h.json)"; done; done
CPD_FM_LDS=20480 bash tools_scripts/trace_ab.sh r05n CPD_UP_HEAD "0"
CPD_FM_LDS=13824 bash tools_scripts/trace_ab.sh r05n13 CPD_UP_HEAD "0"
