#!/bin/bash
# Knob A/B at the final batch size, then a 2-rank launch rehearsal on one GPU.
set -o pipefail
mkdir -p gpurun_out
bash tools_scripts/gpu_env_ab.sh k_down8 CPD_DOWN8_WPB "2 4 1" none || exit 1
bash tools_scripts/gpu_env_ab.sh k_fmwpb CPD_FM_WPB "2 4 1" none || exit 1
CPD_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-pmc \
    > gpurun_out/share2.json 2> gpurun_out/share2.err || { echo "2-rank rehearsal failed"; tail -20 gpurun_out/share2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/share2.json'));print('2 ranks (shared GPU, rehearsal only):', d['n_gpus'], d['value'], d['config']['rows_per_step_per_gpu'])"
