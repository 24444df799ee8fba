#!/bin/bash
# Two SQ counter passes (8 SQ counters each, no tracing domains) over profiles/attn_probe.py,
# reduced to per-kernel means:  gpurun -- 'bash profiles/attn_pmc.sh TAG'
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/attn_pmc_$TAG
mkdir -p "$OUT"
P=(python3 profiles/attn_probe.py --iters 2)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS -f rocpd -d "$OUT/p1" -o run -- "${P[@]}" > "$OUT/p1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32 -f rocpd -d "$OUT/p2" -o run -- "${P[@]}" > "$OUT/p2.log" 2>&1
python3 profiles/rocpd_tools.py pmc "$(find "$OUT/p1" -name '*.db' -print -quit)" "$(find "$OUT/p2" -name '*.db' -print -quit)" > "$OUT/pmc.json"
rm -rf "$OUT/p1" "$OUT/p2"
echo "[attn_pmc] $OUT/pmc.json"
