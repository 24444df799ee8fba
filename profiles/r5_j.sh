#!/bin/bash
# round 5, call j: the split-P relative-key forward normalised by the sum of the same hi + lo P
# (weights sum to 1: the common value component no longer leaks into delta).  Attention kernel
# tests, full-size parity against the same-instance floor, the floor diagnostics at c5 / c1, the
# isolated forward time and c2 / c5 lines: libste.so (new) vs libste_ab.so (previous attention.hip)
source profiles/r5_lib.sh
O=gpurun_out/r5j; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
PYF=(python -u -m pytest -v -s --timeout 900 --timeout-method thread -p no:cacheprovider)
step attn_tests 300 "${PYT[@]}" tests/test_kernels_gpu.py -k "attention or attn" > $O/attn_tests.log 2>&1
step fullsize 900 "${PYF[@]}" tests/test_fullsize_gpu.py > $O/fullsize.log 2>&1
step diag 600 python -u profiles/r5_floor_diag.py c5 > $O/floor_diag.log 2>&1
step probe_new 200 python -u profiles/attn_probe.py --iters 30 > $O/probe_new.json 2>&1
STE_LIB=$AB step probe_old 200 python -u profiles/attn_probe.py --iters 30 > $O/probe_old.json 2>&1
for i in 1 2; do
  step bench_new_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err
  STE_LIB=$AB step bench_old_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_old_$i.json 2> $O/bench_old_$i.err
done
