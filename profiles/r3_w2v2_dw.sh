#!/bin/bash
# round-3: wav2vec2 conv-stack per-clip dW on the 8-phase kernel (STE_GEMM_BATCHED_DW=0: the
# 128x128 kernel) — parity tests, then wav2vec2-base bench lines A/B on one box
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_w2v2_gpu.py -k "batched_dw or w2v or conv or gemm_dw" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_w2v2dw.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --audio-model facebook/wav2vec2-base > gpurun_out/w2dw_on1.json 2>/dev/null
STE_GEMM_BATCHED_DW=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --audio-model facebook/wav2vec2-base > gpurun_out/w2dw_off1.json 2>/dev/null
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --audio-model facebook/wav2vec2-base > gpurun_out/w2dw_on2.json 2>/dev/null
STE_GEMM_BATCHED_DW=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --audio-model facebook/wav2vec2-base > gpurun_out/w2dw_off2.json 2>/dev/null
