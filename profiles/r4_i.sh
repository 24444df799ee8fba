#!/bin/bash
# kernel-time breakdown at HEAD (packed fp32 off): c2 and c5 (bf16), kernel trace + stats only
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r4i/c2 -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r4i/c2_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r4i/c5 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --seconds 30 --freeze none > gpurun_out/r4i/c5_bench.json
find gpurun_out/r4i -name '*kernel_trace.csv' -delete
