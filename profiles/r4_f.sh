#!/bin/bash
mkdir -p gpurun_out
REPS=60 timeout -k 10 280 python -u profiles/det_ln.py > gpurun_out/r4f_ln.log 2>&1; echo "ln rc=$?"
