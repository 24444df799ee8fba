#!/bin/bash
# round 6, call l: the b = 32 per-GPU step (c3's batch at N = 8) under rocprofv3 — where its per-pair
# time exceeds b = 64's — kernel trace + stats, and its dispatch-gap timeline
source profiles/r6_lib.sh
O=gpurun_out/r6l; mkdir -p $O
step profile_b32 900 bash profiles/profile_bench.sh r6b32 --batch 32 > $O/profile_b32.log 2>&1
