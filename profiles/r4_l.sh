#!/bin/bash
# LayerNorm in isolation (c2 rows), then config 5 (30 s clips, full unfreeze) bf16 and --fp8 lines,
# and the c5 bf16 kernel trace, at HEAD
mkdir -p gpurun_out/r4l
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/kernel_timer.py layernorm > gpurun_out/r4l/ln_isolation.txt 2>&1; echo "ln rc=$?"
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > gpurun_out/r4l/c5_bf16.json 2> gpurun_out/r4l/c5_bf16.err; echo "c5 rc=$?"
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > gpurun_out/r4l/c5_fp8.json 2> gpurun_out/r4l/c5_fp8.err; echo "c5fp8 rc=$?"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r4l/c5 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --seconds 30 --freeze none > gpurun_out/r4l/c5_trace_bench.json; echo "trace rc=$?"
find gpurun_out/r4l -name '*kernel_trace.csv' -delete
