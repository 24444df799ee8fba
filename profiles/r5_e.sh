#!/bin/bash
# round 5, call e: the 1,024-thread fp32 text attention backward + compiled dz epilogue spec:
# kernel tests, the loss-derived model tests, then alternated c2 lines precise vs bf16 text backward
source profiles/r5_lib.sh
O=gpurun_out/r5e; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
step kern 600 "${PYT[@]}" -s tests/test_kernels_gpu.py -k "attention_f32 or adamw or gemm" > $O/kern.log 2>&1
step model 600 "${PYT[@]}" -s tests/test_model_gpu.py -k "golden_and_oracle" > $O/model.log 2>&1
for i in 1 2; do
  STE_LIB=$AB STE_TEXT_PRECISE_BWD=1 step bench_p_$i 300 python -u bench.py --no-cpu-baseline --steps 15 > $O/bench_p_$i.json 2> $O/bench_p_$i.err
  STE_LIB=$AB STE_TEXT_PRECISE_BWD=0 step bench_b_$i 300 python -u bench.py --no-cpu-baseline --steps 15 > $O/bench_b_$i.json 2> $O/bench_b_$i.err
done
STE_LIB=$AB STE_TEXT_PRECISE_BWD=1 step prof 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_p -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_p.json 2> $O/prof_p.err
