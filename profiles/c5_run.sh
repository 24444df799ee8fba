#!/bin/bash
# c5 (BASELINE config 5 per-GPU shape: 30 s clips, every layer trainable, b = 64) bench lines in
# bf16 and MX-fp8, then the rocprofv3 kernel stats + PMC traffic of the fp8 line (profile_bench.sh).
set -e -o pipefail
T=${1:-r03}
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/${T}_c5bf16.json 2> gpurun_out/${T}_c5bf16.err
timeout -k 10 300 python3 -u bench.py --seconds 30 --freeze none --fp8 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/${T}_c5fp8.json 2> gpurun_out/${T}_c5fp8.err
bash profiles/profile_bench.sh ${T}_c5fp8 --seconds 30 --freeze none --fp8 > gpurun_out/${T}_c5prof.log 2>&1
