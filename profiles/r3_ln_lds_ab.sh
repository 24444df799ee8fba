#!/bin/bash
# round-3 same-box A/B: LayerNorm backward column sums in registers (in-tree lib) vs in LDS
# (scratch/libste_lds.so), isolated kernel timing and c2 bench lines, interleaved
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ab_ln_reg.txt
STE_LIB=scratch/libste_lds.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ab_ln_lds.txt
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab_reg1.json 2>/dev/null
STE_LIB=scratch/libste_lds.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab_lds1.json 2>/dev/null
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab_reg2.json 2>/dev/null
STE_LIB=scratch/libste_lds.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab_lds2.json 2>/dev/null
