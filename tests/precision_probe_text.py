"""Precision probe of the loss-derived gradients at the golden mini dims (test tooling, imports
oracle/; CPU only).

Question (VERDICT r4 "What's weak" #1, the loss-derived elementwise bound): the HIP path's
loss-derived gradients sit 1.2-2.0 % (worst tensor) from the fp32 oracle, always on the
trainable text layer's attention weights / biases, the token-type row and the embedding
LayerNorm.  The loss gradient there is the difference of the clean and corrupted transcripts'
nearly equal backward passes.  Which rounding points of the HIP path carry that error?

Method: the oracle's step (oracle/ref_model.py) in fp32, and again with bf16 rounding injected
where engine.py / the kernels round, each site behind a flag:
  tdy   text backward dY operands stored bf16: the gradient at every text Linear output (dy2b,
        dzt, dy1b, dqkv: engine._postln_bwd), i.e. what the dX and dW GEMMs read
  tdo   the attention output gradient dO in bf16 (the O-proj dX GEMM's bf16 output)
  tatt  the text attention backward's bf16 MFMA operands: P for dV, dS for dQ / dK
  tdwx  the trained text layers' dW operands X in bf16 (the forward saves the hi halves)
  afa   the audio side as the HIP path runs it, coarsely: every audio Linear output and the audio
        hidden states rounded to bf16 in the forward (the audio encoder's bf16 storage)
  tqk   (round 5) the text attention backward recomputes P from the bf16 q / k copies against the
        fp32 forward's LSE (p = exp(bf16(q)·bf16(k)ᵀ·scale - LSE)): P no longer sums to 1 per row
  (diagnostic, not a flag: tqk_norm = the same with an LSE of the bf16 scores, p summing to 1)
Per-tensor error = ||g - g_fp32|| / ||g_fp32|| over the tensors test_model_gpu.py checks.

    python tests/precision_probe_text.py [--tag nopool] [--sets all]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from kref import bf16_exact  # noqa: E402
from oracle import det_init, ref_model as R  # noqa: E402

GOLDEN = ROOT / "tests" / "golden"
FLAGS = ("tdy", "tdo", "tatt", "tdwx", "afa", "tqk")


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


class _G(torch.autograd.Function):
    """Identity forward; the incoming gradient rounded to bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return bf(g)


class _LinX(torch.autograd.Function):
    """y = x Wᵀ + b whose weight gradient reads bf16(x) (the saved hi half)."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.hb = b is not None
        return F.linear(x, W, b)

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        gW = g2.t() @ bf(x.reshape(-1, x.shape[-1]))
        return g @ W, gW, (g2.sum(0) if ctx.hb else None)


class _TAttn(torch.autograd.Function):
    """Text SDPA (masked rows: zero weights) whose backward rounds P (for dV) and dS (for dQ/dK);
    qk: None (backward P = the forward's), "lse" (recomputed from bf16 q / k against the fp32
    forward's LSE) or "norm" (recomputed from bf16 q / k, normalised)."""

    @staticmethod
    def forward(ctx, q, k, v, add_mask, rowok, qk=None):
        s = q @ k.transpose(-2, -1) / math.sqrt(q.shape[-1])
        if add_mask is not None:
            s = s + add_mask
        pr = torch.softmax(s, -1)
        pb = pr
        if qk is not None:
            sb = bf(q) @ bf(k).transpose(-2, -1) / math.sqrt(q.shape[-1])
            if add_mask is not None:
                sb = sb + add_mask
            pb = torch.exp(sb - torch.logsumexp(s, -1, keepdim=True)) if qk == "lse" else torch.softmax(sb, -1)
        if rowok is not None:
            pr = pr * rowok
            pb = pb * rowok
        o = pr @ v
        ctx.save_for_backward(q, k, v, pb, o)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, pr, o = ctx.saved_tensors
        sc = 1.0 / math.sqrt(q.shape[-1])
        dp = do @ v.transpose(-2, -1)
        ds = pr * (dp - (do * o).sum(-1, keepdim=True))   # delta = dO·O, as the kernels form it
        dv = bf(pr).transpose(-2, -1) @ do
        dsr = bf(ds)
        return dsr @ k * sc, dsr.transpose(-2, -1) @ q * sc, dv, None, None, None


def probe_text_encoder(fl):
    def text_encoder(p, ids, mask, cfg, prefix="text_encoder."):
        B, L = ids.shape
        nz = (ids != cfg.pad_id).int()
        pos_ids = (torch.cumsum(nz, dim=1) * nz).long() + cfg.pad_id
        e = (F.embedding(ids, p[prefix + "embeddings.word_embeddings.weight"], padding_idx=cfg.pad_id)
             + p[prefix + "embeddings.token_type_embeddings.weight"][0]
             + F.embedding(pos_ids, p[prefix + "embeddings.position_embeddings.weight"], padding_idx=cfg.pad_id))
        x = R._ln(p, prefix + "embeddings.LayerNorm", e, cfg.eps)
        add_mask = rowok = None
        if mask is not None:
            add_mask = (1.0 - mask[:, None, None, :].to(x.dtype)) * R.FINFO_MIN
            rowok = (mask.sum(1) > 0).to(x.dtype)[:, None, None, None]
        H, d = cfg.heads, cfg.hidden // cfg.heads
        g = (lambda t: _G.apply(t)) if fl["tdy"] else (lambda t: t)

        def lin(name, t):
            w, b = p[name + ".weight"], p.get(name + ".bias")
            if fl["tdwx"] and w.requires_grad:
                return _LinX.apply(t, w, b)
            return F.linear(t, w, b)

        for i in range(cfg.layers):
            pre = f"{prefix}encoder.layer.{i}."
            qkv = g(torch.cat([lin(pre + "attention.self.query", x), lin(pre + "attention.self.key", x),
                               lin(pre + "attention.self.value", x)], -1))
            q, k, v = (t.reshape(B, L, H, d).transpose(1, 2) for t in qkv.split(cfg.hidden, -1))
            if fl["tatt"] or fl["tqk"] or fl.get("tqk_norm"):
                o = _TAttn.apply(q, k, v, add_mask, rowok,
                                 "lse" if fl["tqk"] else ("norm" if fl.get("tqk_norm") else None))
            else:
                s = q @ k.transpose(-2, -1) / math.sqrt(d)
                if add_mask is not None:
                    s = s + add_mask
                pr = torch.softmax(s, -1)
                if rowok is not None:
                    pr = pr * rowok
                o = pr @ v
            o = o.transpose(1, 2).reshape(B, L, cfg.hidden)
            if fl["tdo"]:
                o = _G.apply(o)
            x = R._ln(p, pre + "attention.output.LayerNorm", g(lin(pre + "attention.output.dense", o)) + x, cfg.eps)
            inter = F.gelu(g(lin(pre + "intermediate.dense", x)))
            x = R._ln(p, pre + "output.LayerNorm", g(lin(pre + "output.dense", inter)) + x, cfg.eps)
        return x
    return text_encoder


def probe_lin(fl, orig):
    def _lin(p, name, x):
        y = orig(p, name, x)
        if fl["afa"] and name.startswith("audio_encoder"):
            y = bf(y) + (y - y.detach()) * 0   # forward rounding, straight-through backward
        return y
    return _lin


def run(meta, z, fl):
    cfg = R.mini_cfg(meta)
    vals = det_init.state_dict_values(R.param_shapes(cfg, spec_augment=False))
    p = {n: torch.from_numpy(bf16_exact(v)).requires_grad_(n in set(meta["trainable"])) for n, v in vals.items()}
    keys = ["input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
            "attention_mask_audio"]
    batch = {k: torch.from_numpy(z[k]) for k in keys}
    te, lin = R.text_encoder, R._lin
    R.text_encoder = probe_text_encoder(fl)
    R._lin = probe_lin(fl, lin)
    try:
        lo, *_ = R.step_loss(p, batch, cfg)
        lo.backward()
    finally:
        R.text_encoder, R._lin = te, lin
    return {n: p[n].grad.double().reshape(-1).clone() for n in meta["with_grad"] if p[n].grad is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="nopool")
    ap.add_argument("--sets", default="all")
    args = ap.parse_args()
    meta = json.loads((GOLDEN / f"model_golden_{args.tag}.json").read_text())
    z = np.load(GOLDEN / f"model_golden_{args.tag}.npz")
    torch.manual_seed(0)
    ref = run(meta, z, {f: False for f in FLAGS})
    sets = {"hip_text_bwd": ["tdy", "tdo", "tatt", "tdwx"], "tdy": ["tdy"], "tdo": ["tdo"], "tatt": ["tatt"],
            "tdwx": ["tdwx"], "afa": ["afa"], "all": list(FLAGS), "all_but_tdy": ["tdo", "tatt", "tdwx", "afa"],
            "all_but_tatt": ["tdy", "tdo", "tdwx", "afa"], "all_but_tdwx": ["tdy", "tdo", "tatt", "afa"],
            "tatt_tdwx_afa": ["tatt", "tdwx", "afa"], "tatt_afa": ["tatt", "afa"], "tdwx_afa": ["tdwx", "afa"],
            "tdy_tdwx_afa": ["tdy", "tdwx", "afa"], "tdy_afa": ["tdy", "afa"], "tdo_tatt_tdwx_afa": ["tdo", "tatt", "tdwx", "afa"],
            "all_but_tqk": ["tdy", "tdo", "tatt", "tdwx", "afa"], "tqk": ["tqk"],
            "all_tqk_norm": ["tdy", "tdo", "tatt", "tdwx", "afa", "tqk_norm"]}
    if args.sets != "all":
        sets = {k: v for k, v in sets.items() if k in args.sets.split(",")}
    for name, on in sets.items():
        g = run(meta, z, {f: f in on for f in FLAGS + ("tqk_norm",)})
        errs = sorted(((float((g[n] - ref[n]).norm() / ref[n].norm()), n) for n in ref if ref[n].norm() > 1e-6),
                      reverse=True)
        print(json.dumps({"tag": args.tag, "set": name, "flags": on, "worst": [(round(e, 5), n) for e, n in errs[:4]],
                          "median": round(errs[len(errs) // 2][0], 5)}), flush=True)


if __name__ == "__main__":
    main()
