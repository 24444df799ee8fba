#!/bin/bash
# round-3 same-box A/B: the c2 bench line with the round-start library (scratch/ste_e557.so, built
# from e557db0) vs HEAD, alternated; relative-key attention isolated (scratch/ste_head.so vs HEAD)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
for i in 1 2; do
  for T in "--frames 499 --batch 64" "--frames 1499 --batch 16"; do
    STE_LIB=scratch/ste_head.so timeout -k 10 60 python3 -u profiles/attn_probe.py $T >> gpurun_out/attn_head.txt
    timeout -k 10 60 python3 -u profiles/attn_probe.py $T >> gpurun_out/attn_new.txt
  done
done
for i in 1 2; do
  STE_LIB=scratch/ste_e557.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/ab_c2_old.json 2>/dev/null
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/ab_c2_new.json 2>/dev/null
done
