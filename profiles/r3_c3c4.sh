#!/bin/bash
# round-3 final tree: config-3 shape at N = 1 (4 x 64 accumulated) and config 4 (alignment head, 5 unfrozen)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --global-batch 256 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3e_c3n1.json 2> gpurun_out/r3e_c3n1.err
timeout -k 10 300 python3 -u bench.py --align --unfreeze 5 --no-cpu-baseline > gpurun_out/r3e_c4.json 2> gpurun_out/r3e_c4.err
