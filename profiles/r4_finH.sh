#!/bin/bash
# last check at the final tree (after the window fix and the edge tests): full GPU suite, smoke(), default bench line
set -e -o pipefail
mkdir -p gpurun_out/r4fh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4fh/tests.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4fh/smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4fh/bench_c2.json 2> gpurun_out/r4fh/bench_c2.err
