#!/bin/bash
# The N = 8 plumbing rehearsal on a 1-GPU box (CPD_BENCH_SHARE_GPU=1: every
# rank on GPU 0, harness collectives over gloo / files; never a number):
# (the search legs are skipped: eight ranks' fscale-0 searches on one card run
# minutes without output)
# (1) the bench's build + search legs at 8 ranks, (2) the end-to-end worker
# leg (--full-build-only: make_cpd_auto per rank, buckets, fifo_auto serving).
#   tools_scripts/rehearsal_8ranks.sh TAG
set -o pipefail
TAG=${1:-r06_rehearsal}
mkdir -p gpurun_out
export CPD_BENCH_SHARE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 8 --steps 3 --warmup 1 --batch 1024 --no-cpu --no-pmc \
    --no-full-build --no-search --queries 100000 > gpurun_out/${TAG}_8ranks_bench.json 2> gpurun_out/${TAG}_8ranks_bench.err \
    || { echo "8-rank bench failed"; tail -30 gpurun_out/${TAG}_8ranks_bench.err; exit 1; }
tail -c 3000 gpurun_out/${TAG}_8ranks_bench.json
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29612 bench.py --gpus 8 --full-build-only > gpurun_out/${TAG}_8ranks_full_build.json \
    2> gpurun_out/${TAG}_8ranks_full_build.err \
    || { echo "8-rank full build failed"; tail -30 gpurun_out/${TAG}_8ranks_full_build.err; exit 1; }
tail -c 3000 gpurun_out/${TAG}_8ranks_full_build.json
