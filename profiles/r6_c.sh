#!/bin/bash
# round 6, call c: PRO2 (all of K-tile 1 staged in the GEMM prologue, before the previous tile's
# epilogue stores) — the bench-plan parity tests on the new default build, then an isolated GEMM
# A/B against the PRO2=0 build (libste_pro0.so) and alternating c2 bench lines
source profiles/r6_lib.sh
O=gpurun_out/r6c; mkdir -p $O
step new_tests 900 python -u -m pytest tests/test_gemm_specs_gpu.py tests/test_plan_equivalence_gpu.py tests/test_fullsize_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/new_tests.log 2>&1
for L in libste libste_pro0; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step probe_$L 300 python -u profiles/gemm_probe.py --iters 30 > $O/probe_$L.jsonl 2>&1
done
for i in 1 2; do
  for L in libste_pro0 libste; do
    STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step bench_${L}_$i 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${L}_$i.json 2> $O/bench_${L}_$i.err
  done
done
