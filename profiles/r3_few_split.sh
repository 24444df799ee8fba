#!/bin/bash
# round-3: few-tile split-K (text encoder N = 768 outputs) parity + isolated timing under the
# three kernel choices, c2 A/B (STE_GEMM_FEW_SPLIT=0), LayerNorm register vs LDS column sums
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "few_tile or dw_splitk or gemm_epilogues or gemm_layouts" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_few.log 2>&1
timeout -k 10 120 python3 -u profiles/gemm_probe.py --text > gpurun_out/text_default.txt
STE_GEMM_MIN_TILES=64 timeout -k 10 120 python3 -u profiles/gemm_probe.py --text > gpurun_out/text_8ph.txt
STE_GEMM_MIN_TILES=64 STE_GEMM_FEW_SPLIT=0 timeout -k 10 120 python3 -u profiles/gemm_probe.py --text > gpurun_out/text_8ph_nosplit.txt
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ab_ln_reg.txt
STE_LIB=scratch/libste_lds.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ab_ln_lds.txt
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/few_on1.json 2>/dev/null
STE_GEMM_FEW_SPLIT=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/few_off1.json 2>/dev/null
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/few_on2.json 2>/dev/null
