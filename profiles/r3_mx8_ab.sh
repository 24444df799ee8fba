#!/bin/bash
# round-3: MX-fp8 Conformer forward GEMMs on the persistent 8-phase kernel (default) vs the
# single-stage gemm_mx8_kernel (STE_MX8_8PH=0): kernel tests, c5-shape fp8 bench lines; LN column
# sums through the workspace vs atomics (isolated)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "mx8 or layernorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mx8.log 2>&1
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln_ws.txt
STE_LN_ATOMIC=1 timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln_atomic.txt
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --seconds 30 --freeze none --fp8 --steps 6 --warmup 2 > gpurun_out/c5fp8_8ph.json 2> gpurun_out/c5fp8_8ph.err
STE_MX8_8PH=0 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --seconds 30 --freeze none --fp8 --steps 6 --warmup 2 > gpurun_out/c5fp8_old.json 2> gpurun_out/c5fp8_old.err
