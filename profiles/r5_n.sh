#!/bin/bash
# round 5, call n: the other workloads at HEAD (c3's per-GPU batch, c3 at N = 1, c4, forward-only
# evaluation), the per-stage timeline at b = 32, and c5 kernel stats + PMC traffic
source profiles/r5_lib.sh
O=gpurun_out/r5n; mkdir -p $O
step b32 300 python -u bench.py --batch 32 --no-cpu-baseline > $O/line_b32.json 2> $O/line_b32.err
step c3n1 400 python -u bench.py --global-batch 256 --no-cpu-baseline > $O/line_c3n1.json 2> $O/line_c3n1.err
step c4 300 python -u bench.py --align --unfreeze 5 --no-cpu-baseline > $O/line_c4.json 2> $O/line_c4.err
step eval 300 python -u bench.py --eval --no-cpu-baseline > $O/line_eval.json 2> $O/line_eval.err
step stages 300 python -u profiles/r5_stage_times.py --batch 32 > $O/stages_b32.json 2> $O/stages_b32.err
step prof_c5 900 bash profiles/profile_bench.sh r5c5 --seconds 30 --freeze none > $O/prof_c5.log 2>&1
cp gpurun_out/prof_r5c5/kernel_stats.csv profiles/r5c5_kernel_stats.csv
cp gpurun_out/prof_r5c5/hbm_traffic.json profiles/r5c5_hbm_traffic.json
