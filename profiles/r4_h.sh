#!/bin/bash
# packed-fp32 off (default build) vs on (scratch_lib/libste_pk.so): determinism + c2 throughput, one box
# scratch_lib/*.so: one-off builds of this tree (packed fp32 on / layernorm.hip variants), not kept
mkdir -p gpurun_out
export REPS=40 MODES=idle,gemm
timeout -k 10 200 python -u profiles/det_ln.py > gpurun_out/r4h_ln.log 2>&1; echo "ln rc=$?"
timeout -k 10 300 python -u profiles/det_kernels.py > gpurun_out/r4h_kernels.log 2>&1; echo "kernels rc=$?" && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_determinism_gpu.py > gpurun_out/r4h_det.log 2>&1; echo "det rc=$?"
for i in 1 2; do
  timeout -k 10 240 python -u bench.py > gpurun_out/r4h_bench_nopk_$i.json 2> gpurun_out/r4h_bench_nopk_$i.err; echo "nopk$i rc=$?"
  STE_LIB=$PWD/scratch_lib/libste_pk.so timeout -k 10 240 python -u bench.py > gpurun_out/r4h_bench_pk_$i.json 2> gpurun_out/r4h_bench_pk_$i.err; echo "pk$i rc=$?"
done
