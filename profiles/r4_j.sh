#!/bin/bash
# DPP / permlane wave reductions (no ds_bpermute) + split-K reduce with all slab loads in flight + relative-key attention VALU cuts vs the previous build (scratch_lib/libste_prev.so,
# one-off, not kept): kernel tests, c2 A/B, then the c2 kernel trace of the new build
mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or pool or align or fbank or loss or l2norm or xattn or gemm or splitk or attention" > gpurun_out/r4j/tests.log 2>&1; echo "tests rc=$?"
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4j/bench_new_$i.json 2> gpurun_out/r4j/bench_new_$i.err; echo "new$i rc=$?"
  STE_LIB=$PWD/scratch_lib/libste_prev.so timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4j/bench_prev_$i.json 2> gpurun_out/r4j/bench_prev_$i.err; echo "prev$i rc=$?"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r4j/c2 -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r4j/c2_trace_bench.json; echo "trace rc=$?"
find gpurun_out/r4j -name '*kernel_trace.csv' -delete
