#!/bin/bash
# round-4 closing run, part B (final tree): LayerNorm in isolation, config-5 bf16 / fp8 lines,
# c5 kernel stats + PMC HBM traffic, the k-major weight-gradient GEMM probe + LDS counters
set -e -o pipefail
mkdir -p gpurun_out/r4l gpurun_out/r4m
timeout -k 10 120 python -u profiles/kernel_timer.py layernorm > gpurun_out/r4l/ln_isolation.txt 2>&1
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > gpurun_out/r4l/c5_bf16.json 2> gpurun_out/r4l/c5_bf16.err
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > gpurun_out/r4l/c5_fp8.json 2> gpurun_out/r4l/c5_fp8.err
bash profiles/profile_bench.sh r4c5 --seconds 30 --freeze none > gpurun_out/prof_r4c5.log 2>&1
bash profiles/r4_m.sh
