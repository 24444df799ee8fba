#!/bin/bash
# round 5, call t: the 8-phase MX-fp8 GEMM with one scale byte per register (A/B library,
# STE_MX8_8PH=1): every epilogue spec, then c5 fp8 lines on the single-stage kernel (shipped) vs
# the fixed 8-phase one, and the fp8 input-gradient A/B on the 8-phase one
source profiles/r5_lib.sh
O=gpurun_out/r5t; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
STE_LIB=$AB STE_MX8_8PH=1 step mx_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "mx8" > $O/mx_tests.log 2>&1
step c5_fp8_ss 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > $O/c5_fp8_ss.json 2> $O/c5_fp8_ss.err
STE_LIB=$AB STE_MX8_8PH=1 step c5_fp8_8ph 400 python -u bench.py --seconds 30 --freeze none --fp8 --no-cpu-baseline > $O/c5_fp8_8ph.json 2> $O/c5_fp8_8ph.err
STE_LIB=$AB STE_MX8_8PH=1 step c5_fp8bwd_8ph 400 python -u bench.py --seconds 30 --freeze none --fp8 --fp8-bwd --no-cpu-baseline > $O/c5_fp8bwd_8ph.json 2> $O/c5_fp8bwd_8ph.err
step c5_bf16 400 python -u bench.py --seconds 30 --freeze none --no-cpu-baseline > $O/c5_bf16.json 2> $O/c5_bf16.err
