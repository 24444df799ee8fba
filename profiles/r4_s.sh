#!/bin/bash
# fbank mel taps read 8 at a time (no serial LDS chain) vs the previous build (DPP pre-emphasis)
# (scratch_lib/libste_prev.so, one-off, not kept): golden tests, isolation timing alternated
mkdir -p gpurun_out/r4s
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fbank" > gpurun_out/r4s/tests.log 2>&1; echo "tests rc=$?"
for i in 1 2 3; do
  timeout -k 10 120 python -u profiles/kernel_timer.py fbank >> gpurun_out/r4s/fbank_new.txt 2>&1; echo "new rc=$?"
  STE_LIB=$PWD/scratch_lib/libste_prev.so timeout -k 10 120 python -u profiles/kernel_timer.py fbank >> gpurun_out/r4s/fbank_prev.txt 2>&1; echo "prev rc=$?"
done
