#!/bin/bash
# round 5, call o: the opt-in MX-fp8 input-gradient GEMMs (engine.fp8_bwd): the MX act-backward
# GEMM test, the full-size c5 parity of fp8 forward vs fp8 forward + backward, the loss-derived
# mini tests with the floor-based bound, and c5 lines bf16 / fp8 / fp8 + fp8 backward
source profiles/r5_lib.sh
O=gpurun_out/r5o; mkdir -p $O
PYF=(python -u -m pytest -v -s --timeout 900 --timeout-method thread -p no:cacheprovider)
step mx_tests 300 "${PYT[@]}" tests/test_kernels_gpu.py -k "mx8" > $O/mx_tests.log 2>&1
step model_tests 400 "${PYF[@]}" tests/test_model_gpu.py -k "golden_and_oracle or random_cotangents" > $O/model_tests.log 2>&1
step fullsize 600 "${PYF[@]}" tests/test_fullsize_gpu.py -k "c5_fp8" > $O/fullsize.log 2>&1
step c5_fp8bwd 400 python -u bench.py --seconds 30 --freeze none --fp8 --fp8-bwd --no-cpu-baseline > $O/c5_fp8bwd.json 2> $O/c5_fp8bwd.err
step c5_fp8 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > $O/c5_fp8.json 2> $O/c5_fp8.err
step c5_bf16 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > $O/c5_bf16.json 2> $O/c5_bf16.err
