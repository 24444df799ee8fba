#!/bin/bash
# round-3: LayerNorm LDS column accumulators (single + pair backward; plain read-add-write of
# lane-private slots) tests + isolated timing, c2 / c5 bf16 / c5 MX-fp8 / wav2vec2-base lines
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ln3.log 2>&1
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/ln3.txt
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/r3_c2.json 2> gpurun_out/r3_c2.err
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3_c5bf16.json 2> gpurun_out/r3_c5bf16.err
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --fp8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3_c5fp8.json 2> gpurun_out/r3_c5fp8.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --audio-model facebook/wav2vec2-base > gpurun_out/r3_w2v2_bench.json 2> gpurun_out/r3_w2v2_bench.err
