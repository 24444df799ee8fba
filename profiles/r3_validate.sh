#!/bin/bash
# round-3 validation: full GPU suite; relative-key attention (new build vs the round-start kernels,
# scratch/ste_head.so); MX-fp8 forward GEMMs in isolation (8-phase vs single-stage kernel) at c5
# rows; c2 bench line
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
for i in 1 2; do
  for T in "--frames 499 --batch 64" "--frames 1499 --batch 16"; do
    STE_LIB=scratch/ste_head.so timeout -k 10 60 python3 -u profiles/attn_probe.py $T >> gpurun_out/attn_head.txt
    timeout -k 10 60 python3 -u profiles/attn_probe.py $T >> gpurun_out/attn_new.txt
  done
done
timeout -k 10 120 python3 -u profiles/gemm_probe.py --mx8 --rows 95936 --iters 10 > gpurun_out/mx8_probe_8ph.txt
STE_MX8_8PH=0 timeout -k 10 120 python3 -u profiles/gemm_probe.py --mx8 --rows 95936 --iters 10 > gpurun_out/mx8_probe_old.txt
timeout -k 10 240 python3 -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
