#!/bin/bash
# round-4 lines of the other workloads at the final tree (one box): c3 at N = 1 (global batch 256),
# c4 (alignment head, 5 + 5 unfrozen), forward-only evaluation, wav2vec2-base raw-waveform encoder
mkdir -p gpurun_out/r4lines
timeout -k 10 400 python -u bench.py --global-batch 256 --no-cpu-baseline > gpurun_out/r4lines/c3n1.json 2>/dev/null; echo "c3 rc=$?"
timeout -k 10 400 python -u bench.py --align --unfreeze 5 --no-cpu-baseline > gpurun_out/r4lines/c4.json 2>/dev/null; echo "c4 rc=$?"
timeout -k 10 400 python -u bench.py --eval --no-cpu-baseline > gpurun_out/r4lines/eval.json 2>/dev/null; echo "eval rc=$?"
timeout -k 10 400 python -u bench.py --audio-model facebook/wav2vec2-base --no-cpu-baseline > gpurun_out/r4lines/w2v2.json 2>/dev/null; echo "w2v2 rc=$?"
