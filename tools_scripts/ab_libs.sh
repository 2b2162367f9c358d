#!/bin/bash
# Interleaved A/B of two library builds on the search workload (one box, one job):
#   tools_scripts/ab_libs.sh TAG LIB_B [reps]   (A = the tree's libcpd.so, B = LIB_B)
TAG=$1; LIBB=$2; REPS=${3:-2}
mkdir -p gpurun_out
out=gpurun_out/${TAG}_libs_ab.jsonl; : > $out
for r in $(seq $REPS); do
  for lib in A B; do
    for fs in 0 0.1; do
      if [ $lib = B ]; then export CPD_LIB=$PWD/$LIBB; else unset CPD_LIB; fi
      timeout -k 10 200 python tools_scripts/search_ab.py --fscale $fs > gpurun_out/${TAG}_one.json 2>> gpurun_out/${TAG}_libs_ab.err || { tail -5 gpurun_out/${TAG}_libs_ab.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_one.json')); d['lib']='$lib'; d['rep']=$r; print(json.dumps(d))" >> $out
      echo "$lib rep$r fscale $fs $(python3 -c "import json; print(json.load(open('gpurun_out/${TAG}_one.json'))['qps'])")"
    done
  done
done
