#!/bin/bash
# round-4 closing run at the final tree (after the lean LayerNorm forward pair): full GPU suite,
# smoke(), the default bench line (CPU baseline included), c2 kernel stats + PMC traffic, c5 lines
set -e -o pipefail
mkdir -p gpurun_out/r4fc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4fc/tests.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fc/smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4fc/bench_c2.json 2> gpurun_out/r4fc/bench_c2.err
bash profiles/profile_bench.sh r4c2f > gpurun_out/r4fc/prof_c2.log 2>&1
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > gpurun_out/r4fc/c5_bf16.json 2> gpurun_out/r4fc/c5_bf16.err
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > gpurun_out/r4fc/c5_fp8.json 2> gpurun_out/r4fc/c5_fp8.err
