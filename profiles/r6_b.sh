#!/bin/bash
# round 6, call b: the packed-fp32 LayerNorm defect re-checked on this toolchain:
# the shipped libste.so (packed fp32 off) vs libste_pk.so (layernorm.hip compiled with packed fp32,
# everything else identical), profiles/det_ln.py beside our GEMM on a second stream
source profiles/r6_lib.sh
O=gpurun_out/r6b; mkdir -p $O
for L in libste libste_pk; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so MODES=idle,gemm REPS=40 step det_ln_$L 300 python -u profiles/det_ln.py > $O/det_ln_$L.log 2>&1
done
