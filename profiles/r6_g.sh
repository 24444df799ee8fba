#!/bin/bash
# round 6, call g: the c2 profile of the round-6 tree (rocprofv3 kernel trace + stats, FETCH_SIZE /
# WRITE_SIZE passes; the per-dispatch trace kept for profiles/r6_timeline.py), then the c5 shape's
# bf16 and MX-fp8 lines
source profiles/r6_lib.sh
O=gpurun_out/r6g; mkdir -p $O
step profile 1000 bash profiles/profile_bench.sh r6c2 > $O/profile.log 2>&1
B=(python -u bench.py --no-cpu-baseline)
step c5_bf16 300 "${B[@]}" --seconds 30 --freeze none --steps 10 --warmup 3 > $O/c5_bf16.json 2> $O/c5_bf16.err
step c5_fp8 300 "${B[@]}" --seconds 30 --freeze none --fp8 --steps 10 --warmup 3 > $O/c5_fp8.json 2> $O/c5_fp8.err
