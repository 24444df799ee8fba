#!/bin/bash
# round 6, call n: relative-key attention — the SQ counters of the round-6 kernels (VALU : MFMA,
# SQ_WAIT_ANY) and an A/B of raised issue priority around every MFMA cluster
# (-DSTE_ATTN_PRIO=1, libste_aprio.so) against the A/B build without it, isolated at c2 and c5 frames
source profiles/r6_lib.sh
O=gpurun_out/r6n; mkdir -p $O
step pmc 300 bash profiles/attn_pmc.sh r6 > $O/pmc.log 2>&1
for i in 1 2; do
  for L in libste_ab libste_aprio; do
    for T in 499 1499; do
      STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step probe_${L}_T${T}_$i 200 python -u profiles/attn_probe.py --frames $T --iters 20 > $O/probe_${L}_T${T}_$i.json 2>&1
    done
  done
done
