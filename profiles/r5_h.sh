#!/bin/bash
# round 5, call h: k-major operands staged from 32-bit offsets with the lane id regenerated (the
# weight-gradient kernel <false,false,0,0> no longer spills: 47 -> 0 VGPRs to scratch, no scratch
# reloads with vmcnt(0) inside its K-loop): GEMM tests, isolated dW shapes at c2 and c5 rows, c2 and
# c5 lines; new libste.so vs libste_ab.so (the previous gemm.hip)
source profiles/r5_lib.sh
O=gpurun_out/r5h; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
step gemmtests 600 "${PYT[@]}" tests/test_kernels_gpu.py tests/test_small_kernels_gpu.py tests/test_reductions_gpu.py tests/test_w2v2_gpu.py -k "gemm or linear or colsum or dw or w2v2" > $O/gemm_tests.log 2>&1
step probe_new 300 python -u profiles/gemm_probe.py --iters 20 --only dw > $O/probe_new.json 2> $O/probe_new.err
STE_LIB=$AB step probe_old 300 python -u profiles/gemm_probe.py --iters 20 --only dw > $O/probe_old.json 2> $O/probe_old.err
step probe_new5 300 python -u profiles/gemm_probe.py --iters 10 --only dw --rows 95936 > $O/probe_new5.json 2> $O/probe_new5.err
STE_LIB=$AB step probe_old5 300 python -u profiles/gemm_probe.py --iters 10 --only dw --rows 95936 > $O/probe_old5.json 2> $O/probe_old5.err
for i in 1 2; do
  step bench_new_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err
  STE_LIB=$AB step bench_old_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_old_$i.json 2> $O/bench_old_$i.err
done
step c5_new 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline --steps 10 --warmup 3 > $O/c5_new.json 2> $O/c5_new.err
STE_LIB=$AB step c5_old 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline --steps 10 --warmup 3 > $O/c5_old.json 2> $O/c5_old.err
