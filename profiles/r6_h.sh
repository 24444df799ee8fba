#!/bin/bash
# round 6, call h: the GEMM-run LayerNorm (EF_LNF) — its bitwise tests against the separate launches
# (fused sites, counter reuse, uneven load, engine forward on / off), the GEMM spec and LayerNorm
# kernel tests, then the c2 step with and without it (A/B library, STE_LN_FUSE), alternated
source profiles/r6_lib.sh
O=gpurun_out/r6h; mkdir -p $O
T=(python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu)
step ln_tests 400 "${T[@]}" tests/test_gemm_ln_gpu.py > $O/ln_tests.log 2>&1
step spec_tests 400 "${T[@]}" tests/test_gemm_specs_gpu.py tests/test_kernels_gpu.py -k "gemm or layernorm or ln_" > $O/spec_tests.log 2>&1
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
for i in 1 2; do
  for F in 0 1; do
    STE_LIB=$AB STE_LN_FUSE=$F step bench_fuse${F}_$i 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_fuse${F}_$i.json 2> $O/bench_fuse${F}_$i.err
  done
done
