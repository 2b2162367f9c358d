#!/bin/bash
# Host sink ceiling on the GPU box: 16 parallel writers of 2 GB each (32 GB,
# about one e2e worker's DOSCPD02 files) into the directory the e2e worker
# writes, buffered and O_DIRECT; then the worker with --discard (rows built
# and copied out of HBM, nothing written) for the GPU + D2H side alone.
set -o pipefail
TAG=${1:-disk}
R=$PWD
W=/tmp/cpd-e2e-sweep
mkdir -p $W/out gpurun_out
for mode in "" "oflag=direct"; do
  rm -f $W/out/p*
  t0=$(date +%s.%N)
  for i in $(seq 0 15); do dd if=/dev/zero of=$W/out/p$i bs=32M count=64 $mode status=none & done
  wait
  t1=$(date +%s.%N)
  echo "dd 16x2GB ${mode:-buffered}: $(echo "$t1 $t0" | awk "{print \$1-\$2}") s" | tee -a $R/gpurun_out/${TAG}_disk.log
done
rm -f $W/out/p*
[ -f $W/g.xy ] || $R/bin/gen_synth --width 1000 --seed 1 --style shuffled --out $W/g > /dev/null || exit 1
for B in 2048 4096; do
  timeout -k 10 300 $R/bin/make_cpd_auto --input $W/g.xy --partmethod div --partkey 8 --workerid 0 \
      --maxworker 8 --outdir $W/out --device 0 --batch $B --write-threads 16 --discard > $W/log 2>&1 \
      || { echo "discard run failed"; tail -5 $W/log; exit 1; }
  echo "discard B=$B $(grep make_cpd_auto-json $W/log)" | tee -a $R/gpurun_out/${TAG}_disk.log
done
df -h $W | tee -a $R/gpurun_out/${TAG}_disk.log
rm -rf $W/out
