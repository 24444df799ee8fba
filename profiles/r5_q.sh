#!/bin/bash
# round 5, call q: bisect the 8-phase MX-fp8 GEMM (current tree, round-4 final 95b5352, its
# introduction 9795849)
source profiles/r5_lib.sh
O=gpurun_out/r5q; mkdir -p $O
step cur 200 python -u profiles/r5_mx8_bisect.py $PWD > $O/cur.json 2>&1
step r4 200 python -u profiles/r5_mx8_bisect.py $PWD/_old_95b5352 > $O/r4.json 2>&1
step r3 200 python -u profiles/r5_mx8_bisect.py $PWD/_old_9795849 > $O/r3.json 2>&1
