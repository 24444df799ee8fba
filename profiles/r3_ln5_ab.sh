#!/bin/bash
# round-3 same-box A/B: LayerNorm backward without column sums at 5 waves per SIMD (gamma read
# where used, 96 VGPRs with spills: scratch/libste_ln5.so) vs HEAD (4 waves, gamma preloaded)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln5_head.txt
STE_LIB=scratch/libste_ln5.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln5_new.txt
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln5_head2.txt
STE_LIB=scratch/libste_ln5.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln5_new2.txt
