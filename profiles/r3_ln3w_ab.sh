#!/bin/bash
# round-3 same-box A/B: single LayerNorm backward with column sums at 3 waves per SIMD (gamma read
# where used, 768 blocks) vs HEAD (gamma preloaded, 180 VGPRs, 2 waves, 512 blocks:
# scratch/libste_head.so); LN tests, isolated timing, c2 and c5-shape lines
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ln3w.log 2>&1
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln3w_new.txt
STE_LIB=scratch/libste_head.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln3w_head.txt
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ln3w_c2_new1.json 2>/dev/null
STE_LIB=scratch/libste_head.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ln3w_c2_head1.json 2>/dev/null
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ln3w_c5_new.json 2>/dev/null
STE_LIB=scratch/libste_head.so timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ln3w_c5_head.json 2>/dev/null
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ln3w_c2_new2.json 2>/dev/null
STE_LIB=scratch/libste_head.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ln3w_c2_head2.json 2>/dev/null
