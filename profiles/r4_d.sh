#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u profiles/det_kernels.py > gpurun_out/r4d_kernels.log 2>&1; echo "rc=$?"
REPS=6 timeout -k 10 300 python -u profiles/det_kernels.py > gpurun_out/r4d_kernels2.log 2>&1; echo "rc=$?"
