#!/bin/bash
# LayerNorm forward pair: lean variant (STE_LN_FWD_PAIR=lean: no row prefetch, gamma/beta re-read
# per row, 127 VGPRs / 4 waves per SIMD) vs default (172 VGPRs / 2 waves): tests, isolation, c2 lines
mkdir -p gpurun_out/r4p
STE_LN_FWD_PAIR=lean timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" > gpurun_out/r4p/tests_lean.log 2>&1; echo "tests rc=$?"
for i in 1 2; do
  timeout -k 10 120 python -u profiles/kernel_timer.py layernorm > gpurun_out/r4p/ln_default_$i.txt 2>&1; echo "ln default rc=$?"
  STE_LN_FWD_PAIR=lean timeout -k 10 120 python -u profiles/kernel_timer.py layernorm > gpurun_out/r4p/ln_lean_$i.txt 2>&1; echo "ln lean rc=$?"
done
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4p/bench_default_$i.json 2>/dev/null; echo "default$i rc=$?"
  STE_LN_FWD_PAIR=lean timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4p/bench_lean_$i.json 2>/dev/null; echo "lean$i rc=$?"
done
