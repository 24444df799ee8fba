#!/bin/bash
# round 4: ordered reductions — determinism + full GPU suite + c2 bench (perf cost of the ordered sums)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_determinism_gpu.py tests/test_checkpoint_gpu.py -v -s --timeout 280 --timeout-method thread > gpurun_out/r4b_det.log 2>&1
echo "det rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1
echo "suite rc=$?"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err
echo "bench rc=$?"
