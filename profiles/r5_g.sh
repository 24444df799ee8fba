#!/bin/bash
# round 5, call g: GEMM epilogues that load R / Z with the next tile's prologue DMA issued behind
# their first two passes' loads (epilogue_8ph_pre, libste.so) vs the round-4 order (libste_ab.so
# built with -DSTE_EPI_PRE=0): GEMM tests, isolated c2 shapes, alternated c2 lines
source profiles/r5_lib.sh
O=gpurun_out/r5g; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
step gemmtests 600 "${PYT[@]}" tests/test_kernels_gpu.py tests/test_small_kernels_gpu.py tests/test_reductions_gpu.py -k "gemm or linear or colsum" > $O/gemm_tests.log 2>&1
step probe_pre 300 python -u profiles/gemm_probe.py --iters 30 > $O/probe_pre.json 2> $O/probe_pre.err
STE_LIB=$AB step probe_nopre 300 python -u profiles/gemm_probe.py --iters 30 > $O/probe_nopre.json 2> $O/probe_nopre.err
for i in 1 2; do
  step bench_pre_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_pre_$i.json 2> $O/bench_pre_$i.err
  STE_LIB=$AB step bench_nopre_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_nopre_$i.json 2> $O/bench_nopre_$i.err
done
