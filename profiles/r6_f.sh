#!/bin/bash
# round 6, call f: the SW-epilogue bias A/B (libste.so: bias loaded after the main loop, 0 spills in
# the <513,*> instantiations; libste_eb.so: the round-5 preload) on the QKV GEMM probe and two
# alternating c2 bench runs each, then the fixed bench-plan tests (plan equivalence at two levels;
# c4 draws with the alignment head's same-instance floor)
source profiles/r6_lib.sh
O=gpurun_out/r6f; mkdir -p $O
for L in libste libste_eb; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step probe_$L 200 python -u profiles/gemm_probe.py --iters 30 --only qkv > $O/probe_$L.jsonl 2>&1
done
for i in 1 2; do
  for L in libste_eb libste; do
    STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step bench_${L}_$i 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${L}_$i.json 2> $O/bench_${L}_$i.err
  done
done
step tests 700 python -u -m pytest tests/test_plan_equivalence_gpu.py "tests/test_fullsize_gpu.py::test_full_size_vs_oracle[c4-d0]" "tests/test_fullsize_gpu.py::test_full_size_vs_oracle[c4-d1]" "tests/test_fullsize_gpu.py::test_full_size_vs_oracle[c4-d2]" "tests/test_fullsize_gpu.py::test_full_size_mean_excess[c4]" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
