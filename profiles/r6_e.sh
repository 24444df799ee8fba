#!/bin/bash
# round 6, call e: the c5 kernel-stats / PMC profile behind DESIGN's fp8 Amdahl statement, then the
# other workloads' lines at the round-6 tree — c3's per-GPU batch (b = 32), c3 at N = 1 (global
# batch 256), c4, forward-only evaluation
source profiles/r6_lib.sh
O=gpurun_out/r6e; mkdir -p $O
step profile_c5 900 bash profiles/profile_bench.sh r6c5 --seconds 30 --freeze none > $O/profile_c5.log 2>&1
B=(python -u bench.py --no-cpu-baseline)
step b32 200 "${B[@]}" --batch 32 > $O/b32.json 2> $O/b32.err
step c3n1 300 "${B[@]}" --global-batch 256 --steps 10 > $O/c3n1.json 2> $O/c3n1.err
step c4 200 "${B[@]}" --align --unfreeze 5 > $O/c4.json 2> $O/c4.err
step eval 200 "${B[@]}" --eval > $O/eval.json 2> $O/eval.err
