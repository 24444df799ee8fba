#!/bin/bash
# round 6, call j: the text forward enqueued after the audio encoder's first layer (Engine.forward;
# the kernel trace showed the main stream idle ~1.5 ms per step while the host enqueued the text
# forward first): model tests, then c2 with and without it (A/B library, STE_TEXT_AFTER_LAYER,
# alternated); then the other workloads' lines at this tree: c5 bf16 / MX-fp8, b = 32, c3 at N = 1,
# c4, forward-only evaluation
source profiles/r6_lib.sh
O=gpurun_out/r6j; mkdir -p $O
step model_tests 400 python -u -m pytest tests/test_model_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/model_tests.log 2>&1
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
for i in 1 2; do
  for F in 0 1; do
    STE_LIB=$AB STE_TEXT_AFTER_LAYER=$F step bench_after${F}_$i 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_after${F}_$i.json 2> $O/bench_after${F}_$i.err
  done
done
B=(python -u bench.py --no-cpu-baseline)
step c5_bf16 240 "${B[@]}" --seconds 30 --freeze none --steps 10 --warmup 3 > $O/c5_bf16.json 2> $O/c5_bf16.err
step c5_fp8 240 "${B[@]}" --seconds 30 --freeze none --fp8 --steps 10 --warmup 3 > $O/c5_fp8.json 2> $O/c5_fp8.err
step b32 150 "${B[@]}" --batch 32 > $O/b32.json 2> $O/b32.err
step c3n1 200 "${B[@]}" --global-batch 256 --steps 10 > $O/c3n1.json 2> $O/c3n1.err
step c4 150 "${B[@]}" --align --unfreeze 5 > $O/c4.json 2> $O/c4.err
step eval 150 "${B[@]}" --eval > $O/eval.json 2> $O/eval.err
