#!/bin/bash
# round-4 closing evidence at HEAD (fbank DPP and the attention A/B options since r4c2f): c2 kernel
# stats + PMC traffic, then the default bench line reading them, and the c5 bf16 line
set -e -o pipefail
mkdir -p gpurun_out/r4fg
bash profiles/profile_bench.sh r4c2h > gpurun_out/r4fg/prof_c2.log 2>&1
cp gpurun_out/prof_r4c2h/kernel_stats.csv profiles/r4c2h_kernel_stats.csv
cp gpurun_out/prof_r4c2h/hbm_traffic.json profiles/r4c2h_hbm_traffic.json
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4fg/bench_c2.json 2> gpurun_out/r4fg/bench_c2.err
timeout -k 10 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > gpurun_out/r4fg/c5_bf16.json 2> gpurun_out/r4fg/c5_bf16.err
