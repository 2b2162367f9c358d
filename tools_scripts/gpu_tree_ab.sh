#!/bin/bash
# Bench A/B of this tree against another checkout built in-tree (e.g. a git
# worktree of the previous round's commit at ./ab_base), alternating, same box.
#   tools_scripts/gpu_tree_ab.sh TAG DIR [rounds] [bench args]
set -o pipefail
TAG=$1; BASE=$2; N=${3:-2}; shift 3
mkdir -p gpurun_out
R=$PWD
for i in $(seq 1 $N); do
  for side in base new; do
    d=$R; [ $side = base ] && d=$R/$BASE
    ( cd $d && timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu --no-pmc --no-search \
        --no-full-build --queries 100000 "$@" ) > gpurun_out/${TAG}_${side}_$i.json 2> gpurun_out/${TAG}_${side}_$i.err \
      || { echo "$side $i failed"; tail -20 gpurun_out/${TAG}_${side}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${side}_$i.json'));print('$side $i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
