#!/bin/bash
# 8-phase kernel threshold for few-tile GEMMs (text O-proj / input gradients at M = 8,192 run on the
# 128x128 kernel below 240 256x256 tiles): STE_GEMM_MIN_TILES=64 vs the default, c2 lines alternated
mkdir -p gpurun_out/r4v
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4v/default_$i.json 2>/dev/null; echo "default$i rc=$?"
  STE_GEMM_MIN_TILES=64 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4v/t64_$i.json 2>/dev/null; echo "t64$i rc=$?"
done
