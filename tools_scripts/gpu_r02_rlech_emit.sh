#!/bin/bash
# Chunked RLE count + deferred emit: GPU parity (incl. driver flow and
# streamed indexes), then bench A/B over CPD_RLE_CH and CPD_EMIT_AT.
set -o pipefail
bash tools_scripts/gpu_env_ab.sh rlech CPD_RLE_CH "32 0 64" tests/test_gpu_parity.py tests/test_gpu_scale_1m.py tests/test_gpu_drivers.py tests/test_gpu_index_stream.py || exit 1
bash tools_scripts/gpu_env_ab.sh emit CPD_EMIT_AT "2 1 0" none
