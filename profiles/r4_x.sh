#!/bin/bash
# forward PV on bf16 P only (STE_ATTN_PLO=0; o_lo still the fp32 O) vs hi + lo P: attention tests
# with their printed errors, full-size parity (all configs), mini parity, isolation timing, c2 lines
mkdir -p gpurun_out/r4x
export PYTHONUNBUFFERED=1
STE_ATTN_PLO=0 timeout -k 10 300 python -u -m pytest -x -s -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "relkey" > gpurun_out/r4x/attn_plo0.log 2>&1; echo "attn plo0 rc=$?"
timeout -k 10 300 python -u -m pytest -x -s -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "relkey" > gpurun_out/r4x/attn_plo1.log 2>&1; echo "attn plo1 rc=$?"
STE_ATTN_PLO=0 timeout -k 10 900 python -u -m pytest -s -q --timeout 800 --timeout-method thread tests/test_fullsize_gpu.py tests/test_model_gpu.py > gpurun_out/r4x/parity_plo0.log 2>&1; echo "parity plo0 rc=$?"
for T in 499 1499; do
  STE_ATTN_PLO=0 timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 --no-bwd >> gpurun_out/r4x/probe_plo0.jsonl 2>/dev/null; echo "probe plo0 $T rc=$?"
  timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 --no-bwd >> gpurun_out/r4x/probe_plo1.jsonl 2>/dev/null; echo "probe plo1 $T rc=$?"
done
for i in 1 2; do
  STE_ATTN_PLO=0 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4x/bench_plo0_$i.json 2>/dev/null; echo "plo0 $i rc=$?"
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4x/bench_plo1_$i.json 2>/dev/null; echo "plo1 $i rc=$?"
done
