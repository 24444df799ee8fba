#!/bin/bash
# what the forward's hi/lo P split (o_lo, for the backward's delta) costs, in isolation, c2 and c5 frames
mkdir -p gpurun_out/r4w
for T in 499 1499; do
  timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 --no-bwd >> gpurun_out/r4w/split.jsonl 2>/dev/null; echo "split $T rc=$?"
  timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 --no-bwd --no-split >> gpurun_out/r4w/nosplit.jsonl 2>/dev/null; echo "nosplit $T rc=$?"
done
