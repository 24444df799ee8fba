#!/bin/bash
# fbank variants (libste_ab.so): frames per wave of a log-mel rewrite (STE_FBANK_FPW, since reverted); round 5 also
# ran STE_FBANK_SN = old / fused statistics variants the same way (profiles/r5w_fbank_ab.txt)
set -e
mkdir -p gpurun_out
for v in 4 8 16 4 8 16; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/libste_ab.so STE_FBANK_FPW=$v timeout -k 10 120 python -u profiles/r5_fbank_bench.py 2>/dev/null | sed "s/^/$v /"
done
