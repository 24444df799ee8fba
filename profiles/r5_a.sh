#!/bin/bash
# round 5, first GPU call: the rel4 forward without the hi/lo P split (row sum over the same rounded
# P, libste.so default) vs the split (STE_ATTN_PLO=1 on libste_ab.so): attention kernel tests, the
# parity suites, then alternated c2 lines
source profiles/r5_lib.sh
O=gpurun_out/r5a; mkdir -p $O
AB=speech_transcript_embeddings_amd/libste_ab.so
step attn 600 "${PYT[@]}" -s tests/test_kernels_gpu.py -k "attention" > $O/attn.log 2>&1
step parity 900 "${PYT[@]}" -s tests/test_fullsize_gpu.py tests/test_model_gpu.py > $O/parity.log 2>&1
for i in 1 2; do
  step bench_new_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err
  STE_LIB=$PWD/$AB STE_ATTN_PLO=1 step bench_plo_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_plo_$i.json 2> $O/bench_plo_$i.err
done
for T in 499 1499; do
  step probe_new_$T 120 python -u profiles/attn_probe.py --frames $T --iters 30 >> $O/probe_new.jsonl 2>> $O/probe.err
  STE_LIB=$PWD/$AB STE_ATTN_PLO=1 step probe_plo_$T 120 python -u profiles/attn_probe.py --frames $T --iters 30 >> $O/probe_plo.jsonl 2>> $O/probe.err
done
