#!/bin/bash
# round-3 scratch measurements: attention kernel tests + isolated timing, GEMM epilogue census
set -e -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or layernorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1
timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd > gpurun_out/abl_lsum.txt
timeout -k 10 60 python3 -u profiles/attn_probe.py > gpurun_out/abl_lsum_bwd.txt
STE_GEMM_CENSUS=gpurun_out/census_c2.json timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --trace-steps 0 > gpurun_out/census_c2_bench.json 2>&1
STE_GEMM_CENSUS=gpurun_out/census_w2v2.json timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --trace-steps 0 --audio-model facebook/wav2vec2-base > gpurun_out/census_w2v2_bench.json 2>&1
STE_LIB=scratch/ste_before.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln_before.txt
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln_after.txt
