#!/bin/bash
# forward PV in fp16 on fp16-rounded P (STE_ATTN_PV16=1, V converted in LDS) vs the hi + lo bf16
# split of P: attention tests with their printed errors, isolation timing, full-size + mini parity,
# c2 lines.  Every step stops the script on failure.
mkdir -p gpurun_out/r4y
export PYTHONUNBUFFERED=1
STE_ATTN_PV16=1 timeout -k 10 300 python -u -m pytest -s -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "relkey or attention" > gpurun_out/r4y/attn_pv16.log 2>&1
rc=$?; echo "attn pv16 rc=$rc"; [ $rc -le 1 ] || exit 1   # 1 = test failures (errors printed), more = crash
for T in 499 1499; do
  STE_ATTN_PV16=1 timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 --no-bwd >> gpurun_out/r4y/probe_pv16.jsonl 2>/dev/null || { echo "probe pv16 $T failed"; exit 1; }
  timeout -k 10 120 python -u profiles/attn_probe.py --frames $T --iters 30 --no-bwd >> gpurun_out/r4y/probe_split.jsonl 2>/dev/null || { echo "probe split $T failed"; exit 1; }
done
echo "probes ok"
STE_ATTN_PV16=1 timeout -k 10 900 python -u -m pytest -s -q --timeout 800 --timeout-method thread tests/test_fullsize_gpu.py tests/test_model_gpu.py > gpurun_out/r4y/parity_pv16.log 2>&1 || { echo "parity pv16 failed"; exit 1; }
echo "parity ok"
for i in 1 2; do
  STE_ATTN_PV16=1 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4y/bench_pv16_$i.json 2>/dev/null || exit 1
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r4y/bench_split_$i.json 2>/dev/null || exit 1
done
echo "bench ok"
