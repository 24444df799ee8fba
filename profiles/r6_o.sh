#!/bin/bash
# round 6, call o: six more seeded draws per full-size config at the final tree (profiles/r6_seed_sweep.py:
# HIP vs the same-instance bf16 floor, per-tensor excess over all audio tensors and all distance tables)
source profiles/r6_lib.sh
O=gpurun_out/r6o; mkdir -p $O
step sweep 1100 python -u profiles/r6_seed_sweep.py --configs c1,c2,c4,c5 --seeds 6 > $O/seed_sweep.jsonl 2> $O/seed_sweep.err
