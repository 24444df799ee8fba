#!/bin/bash
# round 6, call k: the c5 profile (bf16; rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE
# passes) behind DESIGN's fp8 Amdahl statement
source profiles/r6_lib.sh
O=gpurun_out/r6k; mkdir -p $O
step profile_c5 1100 bash profiles/profile_bench.sh r6c5 --seconds 30 --freeze none > $O/profile_c5.log 2>&1
