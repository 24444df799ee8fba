#!/bin/bash
# round-3: few-tile split-K from 40 K-tiles (the text QKV dX back on the 128x128 kernel): tests, c2 A/B
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "few_tile or batched_dw or gemm_layouts" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_few40.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/few40_c2a.json 2>/dev/null
STE_GEMM_FEW_SPLIT=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/few40_off.json 2>/dev/null
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/few40_c2b.json 2>/dev/null
