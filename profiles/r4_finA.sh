#!/bin/bash
# round-4 closing run, part A (final tree): full GPU suite, smoke(), the default bench line (CPU
# baseline included), rocprofv3 kernel stats + PMC HBM traffic of c2 (profile_bench.sh)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_final_tests.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final_smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err
bash profiles/profile_bench.sh r4c2 > gpurun_out/prof_r4c2.log 2>&1
