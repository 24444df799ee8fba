#!/bin/bash
# LayerNorm column-sum backward without dsum on a 4-wave kernel (no dsum accumulators, residual read
# where used, 1024 blocks) vs STE_LN_BWD_DSUM=always (every column-sum launch on the 3-wave dsum
# kernel, round 3): tests both ways, isolation, c5 lines alternated (every layer trainable)
mkdir -p gpurun_out/r4q
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" > gpurun_out/r4q/tests_new.log 2>&1; echo "tests rc=$?"
STE_LN_BWD_DSUM=always timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" > gpurun_out/r4q/tests_always.log 2>&1; echo "tests always rc=$?"
for i in 1 2; do
  timeout -k 10 120 python -u profiles/kernel_timer.py layernorm > gpurun_out/r4q/ln_new_$i.txt 2>&1; echo "ln new rc=$?"
  STE_LN_BWD_DSUM=always timeout -k 10 120 python -u profiles/kernel_timer.py layernorm > gpurun_out/r4q/ln_always_$i.txt 2>&1; echo "ln always rc=$?"
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r4q/c5_new_$i.json 2>/dev/null; echo "c5 new$i rc=$?"
  STE_LN_BWD_DSUM=always timeout -k 10 300 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r4q/c5_always_$i.json 2>/dev/null; echo "c5 always$i rc=$?"
done
