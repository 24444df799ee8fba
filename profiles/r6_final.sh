#!/bin/bash
# round 6, closing call: the whole GPU suite at the final tree with its parity prints (collected by
# profiles/r6_parity.py into profiles/r6_parity.txt), smoke, and the default c2 bench line
source profiles/r6_lib.sh
O=gpurun_out/${R6_OUT:-r6final}; mkdir -p $O
step gpu_tests 1000 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step bench_c2 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err
# the c2 profile of the same tree (rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes), in
# the time left under the call's limit
LEFT=$((1120 - SECONDS))
if [ $LEFT -gt 420 ]; then step profile $LEFT bash profiles/profile_bench.sh ${R6_PROF:-r6c2} > $O/profile.log 2>&1; fi
