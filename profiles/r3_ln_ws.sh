#!/bin/bash
# round-3: LayerNorm column sums through a per-block workspace (deterministic) — kernel tests,
# isolated timing vs the atomic path, attention forward with E staged by DMA (tests), c2 bench
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm or attention or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ln.log 2>&1
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln_ws.txt
STE_LN_ATOMIC=1 timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln_atomic.txt
timeout -k 10 240 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --seconds 30 --freeze none --steps 6 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
