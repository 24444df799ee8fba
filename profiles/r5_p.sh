#!/bin/bash
# round 5, call p: the persistent 8-phase MX kernel's compile-time epilogues at >= 240 tiles
source profiles/r5_lib.sh
O=gpurun_out/r5p; mkdir -p $O
step mx_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "mx8" > $O/mx_tests.log 2>&1
