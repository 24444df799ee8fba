#!/bin/bash
# round-3 same-box A/B of the LayerNorm kernels before (scratch/ste_lnold.so: layernorm.hip at
# bb62cc9) and after the round's next-row-prefetch change (scratch/ste_cur.so), isolated and in the
# c2 step (everything else identical)
set -e -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  STE_LIB=scratch/ste_lnold.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm >> gpurun_out/lnab_old.txt
  STE_LIB=scratch/ste_cur.so timeout -k 10 60 python3 -u profiles/kernel_timer.py layernorm >> gpurun_out/lnab_cur.txt
done
for i in 1 2; do
  STE_LIB=scratch/ste_lnold.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/lnab_c2_old.json 2>/dev/null
  STE_LIB=scratch/ste_cur.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/lnab_c2_cur.json 2>/dev/null
done
