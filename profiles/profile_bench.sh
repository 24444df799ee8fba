#!/bin/bash
# Reproduce the committed profiles/ summaries of a bench.py configuration on the GPU box.
#
#   gpurun -- 'bash profiles/profile_bench.sh r02 [extra bench.py args]'
#
# Three separate rocprofv3 runs of the same command (the guide forbids mixing --pmc with the
# tracing domains, and FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2) do not fit one pass):
#   1. --kernel-trace --stats          -> gpurun_out/prof_TAG/trace/run_kernel_stats.csv
#   2. --pmc FETCH_SIZE                -> gpurun_out/prof_TAG/fetch (rocpd db)
#   3. --pmc WRITE_SIZE                -> gpurun_out/prof_TAG/write (rocpd db)
# then reduces them with profiles/rocpd_tools.py (gfx950 x2 FETCH_SIZE correction) into
# gpurun_out/prof_TAG/{kernel_stats.csv,hbm_traffic.json}; copy those to profiles/TAG_*.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
BENCH=(python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline "$@")
echo "[profile] kernel trace: ${BENCH[*]}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- "${BENCH[@]}" \
    > "$OUT/bench_under_trace.json"
cp "$OUT"/trace/*kernel_stats.csv "$OUT/kernel_stats.csv" 2>/dev/null || \
    find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
echo "[profile] FETCH_SIZE pass"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -f rocpd -d "$OUT/fetch" -o run -- "${BENCH[@]}" > "$OUT/bench_fetch.json"
echo "[profile] WRITE_SIZE pass"
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -f rocpd -d "$OUT/write" -o run -- "${BENCH[@]}" > "$OUT/bench_write.json"
F=$(find "$OUT/fetch" -name "*.db" -print -quit)
W=$(find "$OUT/write" -name "*.db" -print -quit)
python3 profiles/rocpd_tools.py traffic "$F" "$W" > "$OUT/hbm_traffic.json"
rm -rf "$OUT/fetch" "$OUT/write"
echo "[profile] done: $OUT"
