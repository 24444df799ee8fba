#!/bin/bash
# round 6, call i: where the GEMM-run LayerNorm's time goes (profiles/lnf_probe.py at c2 rows): the
# shipped write-through form, plain stores + an agent release per arrival (STE_LNF_MODE=1), and both
# without the LayerNorm rows (the hand-off alone, STE_LNF_SKIP_ROWS)
source profiles/r6_lib.sh
O=gpurun_out/r6i; mkdir -p $O
for L in libste libste_lnf1 libste_lnf0skip libste_lnf1skip; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step probe_$L 200 python -u profiles/lnf_probe.py > $O/probe_$L.jsonl 2>&1
done
