"""Relative-key attention kernels at a BASELINE shape, timed in isolation (HIP events) —
the A/B and PMC harness for the attention work.

    python profiles/attn_probe.py [--batch 64] [--frames 499] [--heads 16] [--iters 20]
    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES ... -- python3 profiles/attn_probe.py --iters 3

Inputs mimic the encoder at random init: q/k/v from the fused [M, 3·1024] projection layout
(row stride 3072, head h at column h·64), w2v-bert's 73-bin distance table, c2's frame count,
a key mask with ragged tails, and values with a large shared component (near-uniform attention)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--frames", type=int, default=499)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-bwd", action="store_true")
    ap.add_argument("--no-split", action="store_true", help="forward without the O_lo (hi + lo P) product")
    a = ap.parse_args()
    from speech_transcript_embeddings_amd import ops
    B, T, H = a.batch, a.frames, a.heads
    D = 64 * H
    M = B * T
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(M, 3 * D, device="cuda", generator=g) * 0.6
    qkv[:, 2 * D:] += torch.randn(B, 1, D, device="cuda", generator=g).expand(B, T, D).reshape(M, D)
    qkv = qkv.bfloat16()
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    mask = torch.ones(B, T, dtype=torch.int32, device="cuda")
    for b in range(0, B, 4):
        mask[b, T - 1 - (b % 37):] = 0
    mask = mask.reshape(-1).contiguous()
    E = (torch.randn(73, 64, device="cuda", generator=g) * 0.3).bfloat16()
    o = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    o_lo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device="cuda")
    do = (torch.randn(M, D, device="cuda", generator=g)).bfloat16()
    dqkv = torch.empty(M, 3 * D, device="cuda", dtype=torch.bfloat16)
    delta = torch.empty(B * H * T, device="cuda")
    dE = torch.zeros(73, 64, device="cuda")
    gwork = torch.empty(B * H * T * 80, device="cuda")

    def fwd():
        ops.attention_fwd(q, k, v, B=B, T=T, H=H, o=o, lse=lse, key_mask=mask, rel_E=E, scale=0.125,
                          o_lo=None if a.no_split else o_lo)

    def bwd():
        ops.attention_bwd(q, k, v, o, lse, do, dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:], B=B, T=T, H=H,
                          delta=delta, key_mask=mask, rel_E=E, scale=0.125, dE=dE, gwork=gwork, o_lo=o_lo)

    fwd()
    if not a.no_bwd:
        bwd()
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("fwd", fwd),) + (() if a.no_bwd else (("bwd", bwd),)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / a.iters, 1)
    fl = 4.0 * B * H * T * T * 64           # QKᵀ + PV (algorithmic, rel term at its minimal cost below)
    fl_rel = 2.0 * B * H * T * 73 * 64
    res["fwd_tflops"] = round((fl + fl_rel) / res["fwd_us"] / 1e6, 1)
    if "bwd_us" in res:
        res["bwd_tflops"] = round((2.5 * fl + 2 * fl_rel) / res["bwd_us"] / 1e6, 1)
    res["shape"] = {"B": B, "T": T, "H": H}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
