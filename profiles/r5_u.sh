#!/bin/bash
# round 5, call u: the whole GPU suite at HEAD (prints kept: the parity numbers of
# profiles/r5_parity.txt) and the smoke entry point
source profiles/r5_lib.sh
O=gpurun_out/r5u; mkdir -p $O
step gpu_tests 1100 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 900 --timeout-method thread > $O/gpu_tests.log 2>&1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
