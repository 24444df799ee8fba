#!/bin/bash
# round-3 A/B: relative-key forward / dQ with E staged by DMA into ring slot 1 (new) vs the
# per-wave E fragment loads (scratch/ste_head.so); then the SQ counters of the new kernels.
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
for i in 1 2; do
  for T in "--frames 499 --batch 64" "--frames 1499 --batch 16"; do
    STE_LIB=scratch/ste_head.so timeout -k 10 60 python3 -u profiles/attn_probe.py $T >> gpurun_out/eslot_head.txt
    timeout -k 10 60 python3 -u profiles/attn_probe.py $T >> gpurun_out/eslot_new.txt
  done
done
timeout -k 10 200 bash profiles/attn_pmc.sh r3new > gpurun_out/attn_pmc.log 2>&1
STE_TEXT_PRECISE=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --trace-steps 0 --steps 3 --warmup 1 > gpurun_out/bench_noprec.json 2> gpurun_out/bench_noprec.err || true
