#!/bin/bash
# relative-key attention in isolation (profiles/attn_probe.py), new build vs scratch_lib/libste_prev.so
# (one-off build of the previous tree, not kept), alternating, c2 and c5 frame counts
mkdir -p gpurun_out/r4k
for i in 1 2; do
  for T in 499 1499; do
    timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 >> gpurun_out/r4k/new_$T.jsonl 2>/dev/null; echo "new $T rc=$?"
    STE_LIB=$PWD/scratch_lib/libste_prev.so timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 >> gpurun_out/r4k/prev_$T.jsonl 2>/dev/null; echo "prev $T rc=$?"
  done
done
