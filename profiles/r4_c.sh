#!/bin/bash
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 200 python -u profiles/det_probe.py --refresh-main > gpurun_out/r4c_det$i.log 2>&1; echo "rc=$?"; done
for i in 4 5 6; do timeout -k 10 200 python -u profiles/det_probe.py --refresh-join > gpurun_out/r4c_det$i.log 2>&1; echo "rc=$?"; done
for i in 7 8 9; do STE_TEXT_STREAM=0 timeout -k 10 200 python -u profiles/det_probe.py --busy > gpurun_out/r4c_det$i.log 2>&1; echo "rc=$?"; done
for i in 10 11 12; do timeout -k 10 200 python -u profiles/det_probe.py > gpurun_out/r4c_det$i.log 2>&1; echo "rc=$?"; done
