#!/bin/bash
# round 5, call s: the 8-phase MX-fp8 GEMM with the scale byte selected by 1 (A/B library,
# STE_MX8_8PH=1): diagnostics and every compile-time epilogue spec
source profiles/r5_lib.sh
O=gpurun_out/r5s; mkdir -p $O
AB=$PWD/speech_transcript_embeddings_amd/libste_ab.so
STE_LIB=$AB STE_MX8_8PH=1 step diag 200 python -u profiles/r5_mx8_diag.py > $O/diag.json 2>&1
STE_LIB=$AB STE_MX8_8PH=1 step mx_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "mx8" > $O/mx_tests.log 2>&1
