#!/bin/bash
# round-3 closing run (after the LN 3-wave, batched-dW changes): full GPU suite, smoke(), the default bench line (CPU baseline included),
# rocprofv3 kernel stats + PMC HBM traffic of c2 (profile_bench.sh r3d)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err
bash profiles/profile_bench.sh r3d > gpurun_out/prof_r3d.log 2>&1
