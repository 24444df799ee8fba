#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 240 python -u profiles/det_ln.py > gpurun_out/r4e_ln.log 2>&1; echo "ln rc=$?"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_kernels_gpu.py::test_attention_relkey" "tests/test_kernels_gpu.py::test_attention_relkey_dE_deterministic" tests/test_checkpoint_gpu.py > gpurun_out/r4e_tests.log 2>&1; echo "tests rc=$?"
