#!/bin/bash
# round-3 final-tree bench lines beside the c2 one: c5 shape bf16 / MX-fp8, wav2vec2-base, eval
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3e_c5bf16.json 2> gpurun_out/r3e_c5bf16.err
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --fp8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3e_c5fp8.json 2> gpurun_out/r3e_c5fp8.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --audio-model facebook/wav2vec2-base > gpurun_out/r3e_w2v2.json 2> gpurun_out/r3e_w2v2.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --eval > gpurun_out/r3e_eval.json 2> gpurun_out/r3e_eval.err
timeout -k 10 200 python3 -u bench.py > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err
