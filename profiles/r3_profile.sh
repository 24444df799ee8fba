#!/bin/bash
# round-3 end-of-work profiles: c2 rocprofv3 kernel stats + PMC HBM traffic (profile_bench.sh r3b),
# the GEMM census of one c2 step, and the cost of the precise text forward (STE_TEXT_PRECISE=0 A/B)
set -e -o pipefail
mkdir -p gpurun_out
bash profiles/profile_bench.sh r3b > gpurun_out/prof_r3b.log 2>&1
STE_GEMM_CENSUS=gpurun_out/census_c2.json timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --trace-steps 1 > gpurun_out/census_c2_bench.json 2>&1
for i in 1 2; do
  STE_TEXT_PRECISE=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/ab_prec0.json 2> gpurun_out/ab_prec0.err
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline >> gpurun_out/ab_prec1.json 2>/dev/null
done
