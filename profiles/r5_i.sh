#!/bin/bash
# round 5, call i: full-size parity against the same-instance bf16 floor (tests/test_fullsize_gpu.py),
# the two-stage text gradient sync (gloo two ranks on one GPU, the RCCL world-1 step), the mini
# model tests, and the per-stage timeline at c3's per-GPU batch with the new text_layers stage
source profiles/r5_lib.sh
O=gpurun_out/r5i; mkdir -p $O
PYF=(python -u -m pytest -v -s --timeout 900 --timeout-method thread -p no:cacheprovider)
step fullsize 1100 "${PYF[@]}" tests/test_fullsize_gpu.py > $O/fullsize.log 2>&1
step dist 400 "${PYT[@]}" tests/test_dist_gpu.py tests/test_rccl_gpu.py tests/test_model_gpu.py > $O/dist_model.log 2>&1
step stages 300 python -u profiles/r5_stage_times.py --batch 32 > $O/stages_b32.json 2> $O/stages_b32.err
