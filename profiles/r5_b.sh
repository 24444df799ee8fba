#!/bin/bash
# round 5, second GPU call: the whole -m gpu suite + smoke at the hygiene tree, the c2 line with its
# CPU baseline, c3's per-GPU shape (--batch 32) and the per-stage backward timeline at b = 32 / 64
# for the data-parallel model of DESIGN §5
source profiles/r5_lib.sh
O=gpurun_out/r5b; mkdir -p $O
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step stages32 300 python -u profiles/r5_stage_times.py --batch 32 > $O/stages_b32.json 2> $O/stages_b32.err
step stages64 300 python -u profiles/r5_stage_times.py --batch 64 > $O/stages_b64.json 2> $O/stages_b64.err
step bench_b32 300 python -u bench.py --batch 32 --no-cpu-baseline > $O/bench_b32.json 2> $O/bench_b32.err
step bench_c2 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
