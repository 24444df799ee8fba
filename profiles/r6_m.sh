#!/bin/bash
# round 6, call m: is the b = 32 step (c3's per-GPU batch at N = 8) host-bound?  Host enqueue time
# vs GPU time per step at b = 2 / 32 / 64 (profiles/host_overhead.py), and the whole step as one
# replayed HIP graph vs eager at b = 32 and 64 (profiles/graph_probe.py); the text-forward enqueue
# point A/B at b = 32 (STE_TEXT_AFTER_LAYER, A/B library)
source profiles/r6_lib.sh
O=gpurun_out/r6m; mkdir -p $O
for b in 2 32 64; do
  step host_b$b 200 python -u profiles/host_overhead.py --batch $b --steps 5 > $O/host_b$b.json 2>&1
done
for b in 32 64; do
  step graph_b$b 300 python -u profiles/graph_probe.py --batch $b --steps 10 > $O/graph_b$b.json 2>&1
done
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
for i in 1 2; do
  for F in 0 1; do
    STE_LIB=$AB STE_TEXT_AFTER_LAYER=$F step b32_after${F}_$i 200 python -u bench.py --batch 32 --no-cpu-baseline > $O/b32_after${F}_$i.json 2> $O/b32_after${F}_$i.err
  done
done
