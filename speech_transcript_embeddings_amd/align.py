"""WordLevelAlignmentModule forward/backward on the HIP kernels (config 4).

ref = /root/reference/training/trainer_unfreeze.py:214-310, invoked at :550-558 on the
positive transcript: text/audio projections -> 4-head text->audio attention with the
audio key-padding mask -> out_proj -> LN(text_hidden + output_projection(.)) ->
confidence MLP (Linear -> ReLU -> Linear) -> scores * text_mask = model.last_alignment_scores
(fed to AlignmentAwareInfoNCE's per-sample weighting, ref:730-734).  The head-averaged
alignment matrix the reference computes is never used, so it is not materialised.
"""
from __future__ import annotations

import torch

from . import _lib, ops
from ._lib import ACT_RELU, ACT_RELU_BWD

BF16, F32 = torch.bfloat16, torch.float32
PRE = "word_level_alignment."


def align_forward(eng, th, thb_pos, ahb, b, L, T, ctx, train, seed, hs):
    s = eng.s
    m = eng.m
    P = m.projection_dim
    nh = m.word_level_alignment.num_heads
    p_drop = m.dropout if train else 0.0
    W = s.w(PRE + "alignment_attention.in_proj_weight")
    bW = s.p(PRE + "alignment_attention.in_proj_bias")
    tp = ops.linear(thb_pos, s.w(PRE + "text_projection.weight"), s.p(PRE + "text_projection.bias"), out_bf16=True)
    ap = ops.linear(ahb, s.w(PRE + "audio_projection.weight"), s.p(PRE + "audio_projection.bias"), out_bf16=True)
    q = ops.linear(tp, W[:P], bW[:P], out_bf16=True)
    kv = ops.linear(ap, W[P:], bW[P:], out_bf16=True)
    probs = eng._e(b * nh * L * T)
    att = eng._e(b * L, P, dtype=BF16)
    ops.align_attn_fwd(q, kv, ctx["a_mask32"], b, L, T, nh, probs, att, drop_p=p_drop, seed=seed)
    o2 = ops.linear(att, s.w(PRE + "alignment_attention.out_proj.weight"),
                    s.p(PRE + "alignment_attention.out_proj.bias"), out_bf16=True)
    y = ops.linear(o2, s.w(PRE + "output_projection.weight"), s.p(PRE + "output_projection.bias"),
                   residual=th[: b * L])
    aligned_b = eng._e(b * L, P, dtype=BF16)
    st = eng._ln(y, PRE + "layer_norm", 1e-5, yb=aligned_b)
    c1 = ops.linear(aligned_b, s.w(PRE + "alignment_confidence.0.weight"), s.p(PRE + "alignment_confidence.0.bias"),
                    act=ACT_RELU, out_bf16=True)
    tmask = eng._e(b * L)
    _lib.call("ste_mask_i64_to_f32", ctx["_tmask_i64"].data_ptr(), tmask.data_ptr(), None, b * L, _lib.stream_ptr())
    scores = ops.linear(c1, s.w(PRE + "alignment_confidence.2.weight"), s.p(PRE + "alignment_confidence.2.bias"),
                        row_scale=tmask)
    hs["align"] = dict(tp=tp, ap=ap, q=q, kv=kv, probs=probs, att=att, o2=o2, y=y, st=st, aligned_b=aligned_b, c1=c1,
                       tmask=tmask, p=p_drop, seed=seed, b=b, L=L, T=T, nh=nh)
    return scores.view(b, L)


def align_backward(eng, d_align, hs, ctx, dth, dah):
    s = eng.s
    m = eng.m
    P = m.projection_dim
    a = hs["align"]
    b, L, T, nh = a["b"], a["L"], a["T"], a["nh"]
    # scores = mlp(aligned) * text_mask  ->  d(mlp out) = d_align * text_mask
    dsc = eng._e(b * L)
    ops.copy2d(dsc, d_align.reshape(b * L))
    _lib.call("ste_scale_rows", dsc.data_ptr(), a["tmask"].data_ptr(), b * L, 1, 1, _lib.stream_ptr())
    # confidence head: Linear(P/2 -> 1) backward through the ReLU, then Linear(P -> P/2)
    c1 = a["c1"]
    dc1 = eng._e(*c1.shape, dtype=BF16)
    g2 = s.g(PRE + "alignment_confidence.2.weight")
    ops.rank1_bwd(dsc, s.p(PRE + "alignment_confidence.2.weight").view(-1), c1, ACT_RELU_BWD, dc1,
                  None if g2 is None else g2.view(-1), s.g(PRE + "alignment_confidence.2.bias"))
    dal = ops.linear_dx(dc1, s.w(PRE + "alignment_confidence.0.weight"))
    eng._dw(dc1, a["aligned_b"], PRE + "alignment_confidence.0.weight")
    eng._db(dc1, PRE + "alignment_confidence.0.bias")
    # LN(text_hidden + output_projection(o2))
    dy = eng._e(b * L, P)
    dyb = eng._e(b * L, P, dtype=BF16)
    eng._ln_bwd(dal, a["y"], a["st"], PRE + "layer_norm", dx=dy, dxb=dyb, dsum=s.g(PRE + "output_projection.bias"))
    ops.axpby(dth[: b * L], dy)
    do2 = ops.linear_dx(dyb, s.w(PRE + "output_projection.weight"), out_bf16=True)
    eng._dw(dyb, a["o2"], PRE + "output_projection.weight")
    datt = ops.linear_dx(do2, s.w(PRE + "alignment_attention.out_proj.weight"), out_bf16=True)
    eng._dw(do2, a["att"], PRE + "alignment_attention.out_proj.weight")
    eng._db(do2, PRE + "alignment_attention.out_proj.bias")
    dq = eng._e(b * L, P, dtype=BF16)
    dkv = eng._e(b * T, 2 * P)
    dsbuf = eng._e(b * nh * L * T)
    ops.align_attn_bwd(a["q"], a["kv"], a["probs"], datt, b, L, T, nh, dsbuf, dq, dkv, drop_p=a["p"], seed=a["seed"])
    W = s.w(PRE + "alignment_attention.in_proj_weight")
    gW = s.g(PRE + "alignment_attention.in_proj_weight")
    gB = s.g(PRE + "alignment_attention.in_proj_bias")
    dtp = ops.linear_dx(dq, W[:P], out_bf16=True)
    if gW is not None:
        ops.linear_dw(dq, a["tp"], out=gW[:P], beta=1.0, ws=eng.ws)
        ops.colsum(dq, gB[:P])
    dkvb = ops.cast_bf16(dkv, eng._e(b * T, 2 * P, dtype=BF16))
    dap = ops.linear_dx(dkvb, W[P:], out_bf16=True)
    if gW is not None:
        ops.linear_dw(dkvb, a["ap"], out=gW[P:], beta=1.0, ws=eng.ws)
        ops.colsum(dkv, gB[P:])
    ops.linear_dx(dtp, s.w(PRE + "text_projection.weight"), out=dth[: b * L], beta=1.0)
    eng._dw(dtp, ctx["_thb"][: b * L], PRE + "text_projection.weight")
    eng._db(dtp, PRE + "text_projection.bias")
    ops.linear_dx(dap, s.w(PRE + "audio_projection.weight"), out=dah, beta=1.0)
    eng._dw(dap, ctx["_ahb"], PRE + "audio_projection.weight")
    eng._db(dap, PRE + "audio_projection.bias")


