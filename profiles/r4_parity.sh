#!/bin/bash
# round 4: parity tests with bf16-exact test weights (full size + mini), printed measurements
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_fullsize_gpu.py tests/test_model_gpu.py -v -s --timeout 900 --timeout-method thread > gpurun_out/r4_parity.log 2>&1
echo "rc=$?"
