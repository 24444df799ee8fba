#!/bin/bash
# GEMM tile groups of 16 m-tiles (scratch_lib/libste_g16.so: this tree built with
# -DSTE_TILE_GROUP=16, one-off, not kept) vs the default 8: c2 GEMMs in isolation, then c2 bench
# lines alternated
mkdir -p gpurun_out/r4o
export TMPDIR=/tmp
G16=$PWD/scratch_lib/libste_g16.so
timeout -k 10 200 python -u profiles/gemm_probe.py --iters 10 > gpurun_out/r4o/gemm_new.jsonl 2>&1; echo "probe new rc=$?"
STE_LIB=$G16 timeout -k 10 200 python -u profiles/gemm_probe.py --iters 10 > gpurun_out/r4o/gemm_g16.jsonl 2>&1; echo "probe g16 rc=$?"
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4o/bench_new_$i.json 2>/dev/null; echo "new$i rc=$?"
  STE_LIB=$G16 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4o/bench_g16_$i.json 2>/dev/null; echo "g16$i rc=$?"
done
