#!/bin/bash
# LayerNorm backward-pair determinism under a concurrent GEMM stream: control vs two compile variants
# scratch_lib/*.so: one-off builds of this tree (packed fp32 on / layernorm.hip variants), not kept
mkdir -p gpurun_out
export REPS=40 MODES=idle,gemm
timeout -k 10 200 python -u profiles/det_ln.py > gpurun_out/r4g_ctl.log 2>&1; echo "ctl rc=$?"
STE_LIB=$PWD/scratch_lib/libste_nopk.so timeout -k 10 200 python -u profiles/det_ln.py > gpurun_out/r4g_nopk.log 2>&1; echo "nopk rc=$?"
STE_LIB=$PWD/scratch_lib/libste_smem.so timeout -k 10 200 python -u profiles/det_ln.py > gpurun_out/r4g_smem.log 2>&1; echo "smem rc=$?"
