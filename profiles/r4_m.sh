#!/bin/bash
# weight-gradient GEMMs (k-major x k-major) at c5 rows in isolation vs hipBLASLt, then LDS / wait
# counters of the dW and of a k-contiguous dX GEMM (one PMC pass, SQ counters only)
mkdir -p gpurun_out/r4m
export TMPDIR=/tmp
timeout -k 10 200 python -u profiles/gemm_probe.py --rows 95936 --iters 10 --only dw > gpurun_out/r4m/dw_c5.jsonl 2>&1; echo "dw rc=$?"
timeout -k 10 200 python -u profiles/gemm_probe.py --rows 31936 --iters 10 > gpurun_out/r4m/gemm_c2.jsonl 2>&1; echo "c2 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES -f csv -d gpurun_out/r4m/pmc -o run -- python3 profiles/gemm_probe.py --rows 95936 --iters 3 --only dw_ffn > gpurun_out/r4m/pmc_bench.txt 2>&1; echo "pmc rc=$?"
