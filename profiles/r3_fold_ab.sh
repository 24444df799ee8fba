#!/bin/bash
# round-3 A/B: relative-key forward with the running max folded into the off-band constant
# (STE_ATTN_FOLD=1, default) vs without; cost of the precise text forward (STE_TEXT_PRECISE=0).
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
for i in 1 2; do
  STE_ATTN_FOLD=0 timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd >> gpurun_out/fold0.txt
  timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd >> gpurun_out/fold1.txt
  STE_ATTN_FOLD=0 timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd --frames 1499 --batch 16 >> gpurun_out/fold0.txt
  timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd --frames 1499 --batch 16 >> gpurun_out/fold1.txt
done
for i in 1 2; do
  STE_TEXT_PRECISE=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --trace-steps 0 >> gpurun_out/bench_noprec.json 2>/dev/null
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --trace-steps 0 >> gpurun_out/bench_prec.json 2>/dev/null
done
