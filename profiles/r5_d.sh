#!/bin/bash
# round 5, call d: cost of the precise text backward.  Alternated c2 lines with STE_TEXT_PRECISE_BWD=1
# (fp32 attention backward, split dY / dW operands) and =0 (bf16 backward), both on libste_ab.so
# (the Python switch is read under the A/B library only); then kernel stats of the precise mode
source profiles/r5_lib.sh
O=gpurun_out/r5d; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
for i in 1 2; do
  STE_LIB=$AB STE_TEXT_PRECISE_BWD=1 step bench_p_$i 300 python -u bench.py --no-cpu-baseline --steps 15 > $O/bench_p_$i.json 2> $O/bench_p_$i.err
  STE_LIB=$AB STE_TEXT_PRECISE_BWD=0 step bench_b_$i 300 python -u bench.py --no-cpu-baseline --steps 15 > $O/bench_b_$i.json 2> $O/bench_b_$i.err
done
STE_LIB=$AB STE_TEXT_PRECISE_BWD=1 step prof 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_p -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_p.json 2> $O/prof_p.err
STE_LIB=$AB STE_TEXT_PRECISE_BWD=0 step prof 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_b -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_b.json 2> $O/prof_b.err
