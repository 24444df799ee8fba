#!/bin/bash
# round 5, call m: closing c2 evidence at HEAD — kernel stats + PMC traffic (profile_bench.sh),
# the default bench line reading them (with the CPU baseline), and the c5 bf16 / fp8 lines
source profiles/r5_lib.sh
O=gpurun_out/r5m; mkdir -p $O
step prof_c2 900 bash profiles/profile_bench.sh r5c2 > $O/prof_c2.log 2>&1
cp gpurun_out/prof_r5c2/kernel_stats.csv profiles/r5c2_kernel_stats.csv
cp gpurun_out/prof_r5c2/hbm_traffic.json profiles/r5c2_hbm_traffic.json
step bench_c2 400 python3 -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
step c5_bf16 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > $O/c5_bf16.json 2> $O/c5_bf16.err
step c5_fp8 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > $O/c5_fp8.json 2> $O/c5_fp8.err
