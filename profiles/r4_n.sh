#!/bin/bash
# L2-aware tile raster (4 m-tiles x 8-wide n-blocks for N >= 2,048) vs the round-3 order
# (scratch_lib/libste_r3raster.so: this tree built with -DSTE_RASTER_R3, one-off, not kept):
# c2 GEMMs in isolation, FETCH_SIZE of the same, then c2 bench lines alternated
mkdir -p gpurun_out/r4n
export TMPDIR=/tmp
R3=$PWD/scratch_lib/libste_r3raster.so
timeout -k 10 200 python -u profiles/gemm_probe.py --iters 10 > gpurun_out/r4n/gemm_new.jsonl 2>&1; echo "probe new rc=$?"
STE_LIB=$R3 timeout -k 10 200 python -u profiles/gemm_probe.py --iters 10 > gpurun_out/r4n/gemm_r3.jsonl 2>&1; echo "probe r3 rc=$?"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/r4n/fetch_new -o run -- python3 profiles/gemm_probe.py --iters 2 > /dev/null 2>&1; echo "fetch new rc=$?"
STE_LIB=$R3 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/r4n/fetch_r3 -o run -- python3 profiles/gemm_probe.py --iters 2 > /dev/null 2>&1; echo "fetch r3 rc=$?"
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4n/bench_new_$i.json 2>/dev/null; echo "new$i rc=$?"
  STE_LIB=$R3 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4n/bench_r3_$i.json 2>/dev/null; echo "r3$i rc=$?"
done
