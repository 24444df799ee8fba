"""Characterise the 8-phase MX-fp8 GEMM's wrong products (run with STE_LIB=.../libste_ab.so
STE_MX8_8PH=1): plain bf16-out epilogue at 252 tiles, against the dequantised fp64 product and
variants that would match a specific fault (scales ignored / taken from another row or k-block,
k-halves of a 128-fp8 K-tile swapped, 32-B chunks swapped)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from speech_transcript_embeddings_amd import ops  # noqa: E402


def deq(q, sc, use_scale=True):
    v = q.view(torch.float8_e4m3fn).double()
    if not use_scale:
        return v
    e = sc.long().repeat_interleave(32, dim=1) - 127
    return v * torch.pow(2.0, e.double())


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def corr(a, b):
    a, b = a.flatten() - a.mean(), b.flatten() - b.mean()
    return (a @ b / (a.norm() * b.norm())).item()


torch.manual_seed(10)
M, N, K = 16000, 1024, 1024
res = {}
for case in ("random", "unit_scales"):
    x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
    xq, wq = ops.mx8_quant(x), ops.mx8_quant(w)
    if case == "unit_scales":   # every scale byte 127 (2^0): a fault in the scale path cannot show
        xq[1].fill_(127)
        wq[1].fill_(127)
    y = ops.linear_mx8(xq, wq, out_bf16=True).double()
    ref = deq(*xq) @ deq(*wq).T
    r = {"rel": rel(y, ref), "corr": corr(y, ref)}
    xv, wv = deq(*xq), deq(*wq)
    # k-halves of each 128-k tile swapped on one operand
    def swap_halves(t, blk=128, part=64):
        t = t.view(t.shape[0], -1, blk // part, part)
        return t.flip(2).reshape(t.shape[0], -1)
    r["corr_swapA_halves"] = corr(y, swap_halves(xv) @ wv.T)
    r["corr_swap32"] = corr(y, swap_halves(xv, 64, 32) @ wv.T)
    r["corr_noscale"] = corr(y, deq(*xq, False) @ deq(*wq, False).T)
    r["first_tile_rel"] = rel(y[:256, :256], ref[:256, :256])
    r["row_rel_first5"] = [rel(y[i], ref[i]) for i in range(5)]
    r["ratio_median"] = (y / ref).median().item()
    res[case] = r
print(json.dumps(res))
