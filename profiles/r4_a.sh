#!/bin/bash
# round 4, first GPU call: full GPU suite (new RCCL world-1 + SpecAugment host-length tests) and a
# c2 bench line at the round-start kernels
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
