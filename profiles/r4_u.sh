#!/bin/bash
# the ordered-reduction GPU tests, then the other workloads' lines
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_reductions_gpu.py > gpurun_out/r4t_reductions.log 2>&1; echo "reductions rc=$?"
bash profiles/r4_lines.sh
