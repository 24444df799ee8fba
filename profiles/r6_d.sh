#!/bin/bash
# round 6, call d: the fixed bench-plan tests (plan equivalence at two levels; c4 draws with the
# alignment head's same-instance floor), then the c2 profile of the round-6 tree: rocprofv3 kernel
# trace + stats and the FETCH_SIZE / WRITE_SIZE passes (profiles/profile_bench.sh), kept with the
# per-dispatch trace for the timeline analysis (profiles/r6_timeline.py)
source profiles/r6_lib.sh
O=gpurun_out/r6d; mkdir -p $O
step tests 900 python -u -m pytest tests/test_plan_equivalence_gpu.py "tests/test_fullsize_gpu.py::test_full_size_vs_oracle[c4-d0]" "tests/test_fullsize_gpu.py::test_full_size_vs_oracle[c4-d1]" "tests/test_fullsize_gpu.py::test_full_size_vs_oracle[c4-d2]" "tests/test_fullsize_gpu.py::test_full_size_mean_excess[c4]" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests.log 2>&1
step profile 1100 bash profiles/profile_bench.sh r6c2 > $O/profile.log 2>&1
