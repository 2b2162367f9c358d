set -o pipefail
W=/tmp/cpd-e2e-sweep
mkdir -p $W/out gpurun_out
[ -f $W/g.xy ] || ./bin/gen_synth --width 1000 --seed 1 --style shuffled --out $W/g > /dev/null || exit 1
CPD_TRACE=1 timeout -k 10 300 ./bin/make_cpd_auto --input $W/g.xy --partmethod div --partkey 8 --workerid 0 --maxworker 8 --outdir $W/out --device 0 --discard > gpurun_out/r04ah_trace.log 2>&1 || { tail -5 gpurun_out/r04ah_trace.log; exit 1; }
grep -E "\[cpd\] graph|make_cpd_auto-json" gpurun_out/r04ah_trace.log | cut -c1-400
