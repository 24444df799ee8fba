"""Precision probe of the alignment head's gradients at the golden mini dims (test tooling,
imports oracle/; CPU only).

Question: test_model_gpu.py::test_backward_random_cotangents[align] puts
word_level_alignment.text_projection.bias at 1.12 % from the fp32 oracle (the other tensors
< 0.9 %).  Which of the HIP path's bf16 rounding points in the head (align.py) carries it?

Method: the oracle's forward with the test's random cotangents (seed 11), the alignment head
(oracle/ref_model.py word_level_alignment, ref:250-310) re-stated with bf16 rounding injected
where align.py rounds, each point behind a flag:
  fwd   forward storage: text/audio hidden (GEMM A operands), tp, ap, q, k/v, att, o2, aligned, c1
  dc1   confidence MLP hidden gradient (rank1_bwd's bf16 dc1)
  dy    LN backward dY operand of the output projection GEMMs (dyb)
  do2   out_proj backward operand (do2, bf16 output of the dX GEMM)
  datt  attention output gradient (bf16)
  dq    query gradient (align_attn_bwd's bf16 dq)
  dtp   text projection gradient (bf16 output of the dX GEMM, read by the dX / dW GEMMs and the
        bias column sum)
Per-tensor error = ||g - g_fp32|| / ||g_fp32|| over the head's parameters.

    python tests/precision_probe_align.py [--sets all]
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
FLAGS = ("fwd", "dc1", "dy", "do2", "datt", "dq", "dtp")
# forward storage sites (each also switched on by "fwd")
FSITES = ("th", "ah", "tp", "ap", "q", "kv", "att", "o2", "al", "c1")


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


class _Q(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, f, b):
        ctx.b = b
        return bf(x) if f else x.clone()

    @staticmethod
    def backward(ctx, g):
        return (bf(g) if ctx.b else g), None, None


def q_(x, f=False, b=False):
    return _Q.apply(x, bool(f), bool(b)) if (f or b) else x


def probe_alignment(fl, gate_store):
    """gate_store["gate"]: the fp32 run's ReLU gate of the confidence MLP, applied in every rounded
    run (as test_model_gpu.py re-runs the oracle with the HIP path's gate): a rounding that flips a
    unit near zero would move a whole gradient row and hide the rounding-level error."""
    fs = set(fl.get("fsites", FSITES if fl["fwd"] else ()))

    def fw_(site):
        return site in fs

    def word_level_alignment(p, pre, text_h, audio_h, text_mask, audio_mask, heads):
        def lin(name, x):
            return F.linear(x, p[pre + name + ".weight"], p.get(pre + name + ".bias"))
        tp = q_(lin("text_projection", q_(text_h, fw_("th"))), fw_("tp"), fl["dtp"])
        ap = q_(lin("audio_projection", q_(audio_h, fw_("ah"))), fw_("ap"))
        B, L, E = tp.shape
        S = ap.shape[1]
        W = p[pre + "alignment_attention.in_proj_weight"]
        bW = p[pre + "alignment_attention.in_proj_bias"]
        qq = q_(F.linear(tp, W[:E], bW[:E]), fw_("q"), fl["dq"])
        k = q_(F.linear(ap, W[E:2 * E], bW[E:2 * E]), fw_("kv"))
        v = q_(F.linear(ap, W[2 * E:], bW[2 * E:]), fw_("kv"))
        d = E // heads
        qq = qq.view(B, L, heads, d).transpose(1, 2)
        k = k.view(B, S, heads, d).transpose(1, 2)
        v = v.view(B, S, heads, d).transpose(1, 2)
        s = (qq @ k.transpose(-2, -1)) / math.sqrt(d)
        if audio_mask is not None:
            s = s.masked_fill((1.0 - audio_mask).bool()[:, None, None, :], float("-inf"))
        w = torch.softmax(s, dim=-1)
        o = q_((w @ v).transpose(1, 2).reshape(B, L, E), fw_("att"), fl["datt"])
        o2 = q_(lin("alignment_attention.out_proj", o), fw_("o2"), fl["do2"])
        y = text_h + q_(lin("output_projection", o2), False, fl["dy"])
        aligned = q_(R._ln(p, pre + "layer_norm", y), fw_("al"))
        z1 = lin("alignment_confidence.0", aligned)
        if "gate" not in gate_store:
            gate_store["gate"] = (z1.detach() > 0).float()
        c1 = q_(z1 * gate_store["gate"].view(z1.shape), fw_("c1"), fl["dc1"])
        sc = lin("alignment_confidence.2", c1).squeeze(-1)
        if text_mask is not None:
            sc = sc * text_mask
        return sc
    return word_level_alignment


def run(meta, z, fl, gate_store):
    cfg = R.mini_cfg(meta)
    vals = det_init.state_dict_values(R.param_shapes(cfg, spec_augment=False))
    p = {n: torch.from_numpy(bf16_exact(v)).requires_grad_(n in set(meta["trainable"])) for n, v in vals.items()}
    keys = ["input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
            "attention_mask_audio"]
    bc = {k: torch.from_numpy(z[k]) for k in keys}
    wla = R.word_level_alignment
    R.word_level_alignment = probe_alignment(fl, gate_store)
    try:
        outs = [o for o in R.compute_pos_neg_embeddings(p, bc, cfg) if o is not None]
    finally:
        R.word_level_alignment = wla
    g = torch.Generator().manual_seed(11)
    cots = [torch.randn(o.shape, generator=g) for o in outs]
    torch.autograd.backward(outs, cots)
    return {n: p[n].grad.double().clone() for n in p if n.startswith("word_level_alignment.") and p[n].grad is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="all")
    args = ap.parse_args()
    meta = json.loads((GOLDEN / "model_golden_align.json").read_text())
    z = np.load(GOLDEN / "model_golden_align.npz")
    gs = {}
    ref = run(meta, z, {f: False for f in FLAGS}, gs)
    sets = {"hip": list(FLAGS), **{f"hip minus {f}": [x for x in FLAGS if x != f] for f in FLAGS},
            **{f"only {f}": [f] for f in FLAGS},
            "bwd": [x for x in FLAGS if x != "fwd"],
            "bwd minus dq, dtp": ["dc1", "dy", "do2", "datt"],
            "bwd minus dtp": ["dc1", "dy", "do2", "datt", "dq"],
            "bwd minus datt, dq, dtp": ["dc1", "dy", "do2"],
            **{f"bwd + fwd {st}": [x for x in FLAGS if x != "fwd"] + [f"f:{st}"] for st in FSITES},
            "hip minus dq, dtp": ["fwd", "dc1", "dy", "do2", "datt"],
            "hip minus dtp": ["fwd", "dc1", "dy", "do2", "datt", "dq"]}
    if args.sets != "all":
        sets = {k: v for k, v in sets.items() if k in args.sets.split(";")}
    for name, on in sets.items():
        fl = {f: f in on for f in FLAGS}
        if any(x.startswith("f:") for x in on):
            fl["fsites"] = tuple(x[2:] for x in on if x.startswith("f:"))
        g = run(meta, z, fl, gs)
        errs = sorted(((float((g[n] - ref[n]).norm() / ref[n].norm()), n.replace("word_level_alignment.", ""))
                       for n in ref if ref[n].norm() > 1e-6), reverse=True)
        print(json.dumps({"set": name, "worst": [(round(e, 5), n) for e, n in errs[:3]]}), flush=True)


if __name__ == "__main__":
    main()
