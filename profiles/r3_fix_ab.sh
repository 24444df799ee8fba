#!/bin/bash
# round-3 same-box A/B: HEAD (LayerNorm backward one row in flight again + compile-time epilogues
# for the precise text QKV / FFN-in GEMMs) vs the library before those two (scratch/ste_cur.so)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm or gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_fix.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_fix_model.log 2>&1
timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm > gpurun_out/fix_ln.txt
for i in 1 2; do
  STE_LIB=scratch/ste_cur.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/fix_c2_cur.json 2>/dev/null
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/fix_c2_new.json 2>/dev/null
done
