#!/bin/bash
# round 5, call k: the split-P forward's LSE from the same MFMA row sum (the exact-p VALU sum
# dropped): attention kernel tests, full-size parity vs the same-instance floor, the isolated
# forward and c2 lines against libste_ab.so (round-5 start attention.hip)
source profiles/r5_lib.sh
O=gpurun_out/r5k; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
PYF=(python -u -m pytest -v -s --timeout 900 --timeout-method thread -p no:cacheprovider)
step attn_tests 300 "${PYT[@]}" tests/test_kernels_gpu.py -k "attention or attn" > $O/attn_tests.log 2>&1
step fullsize 900 "${PYF[@]}" tests/test_fullsize_gpu.py > $O/fullsize.log 2>&1
for i in 1 2; do
  step probe_new_$i 200 python -u profiles/attn_probe.py --iters 30 > $O/probe_new_$i.json 2>&1
  STE_LIB=$AB step probe_old_$i 200 python -u profiles/attn_probe.py --iters 30 > $O/probe_old_$i.json 2>&1
done
for i in 1 2; do
  step bench_new_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err
  STE_LIB=$AB step bench_old_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_old_$i.json 2> $O/bench_old_$i.err
done
