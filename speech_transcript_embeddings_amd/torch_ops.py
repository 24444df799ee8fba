"""PyTorch custom operators over the libste.so C ABI (torch.library, namespace `ste::`).

SURVEY §8(b)'s custom-op layer: each op is a schema'd `torch.ops.ste.*` operator whose
implementation is the HIP kernel behind include/ste.h (launched on the current stream through
ops.py), with a fake (meta) implementation for shape propagation and, where the reference's op
is differentiable, an autograd formula registered with torch.library.register_autograd whose
backward is again a HIP kernel.  They let code outside this package build the step op by op
(tests/test_torch_ops_gpu.py drives the reference's _forward() body, trainer_unfreeze.py:1068-1081,
through them); the fused training step itself calls the C ABI directly (engine.py, train.py).

    ste::fbank(wav, lengths, t_max, pad_value, mask_mode) -> (features, mask)
        SeamlessM4TFeatureExtractor + custom_collate_fn (ref :856-866, :880-921)
    ste::linear(x, weight, bias?) -> y                       nn.Linear, bf16 MFMA / fp32 accumulate
    ste::layer_norm(x, weight, bias, eps) -> (y, mean, rstd) nn.LayerNorm
    ste::attention(q, k, v, key_mask?, rel_E?, scale, rel_left, rel_right) -> (o, lse, o_lo)
        Wav2Vec2BertSelfAttention relative_key core (tf:…wav2vec2_bert…:229-337) / SDPA
    ste::pair_loss(s_pos, s_neg, alignment_scores?, temperature, alignment_weight, corrupt_gamma) -> loss
        AlignmentAwareInfoNCE (ref :702-742)
    ste::adamw_(p!, g, m!, v!, p_bf16!, lr, beta1, beta2, eps, weight_decay, step, sumsq?, max_norm)
        AdamW.step with clip_grad_norm_'s coefficient folded in (ref :1108-1110)

Every op fails loudly (SteError) without the HIP library; there is no CPU implementation.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from . import _lib, ops

BF16, F32 = torch.bfloat16, torch.float32


def _bf16(t: Tensor) -> Tensor:
    """bf16 contiguous 2-D operand (fp32 inputs cast on the ste cast kernel)."""
    t = t.contiguous()
    if t.dtype == BF16:
        return t
    if t.dtype != F32:
        raise TypeError(f"ste ops take fp32 or bf16 tensors, got {t.dtype}")
    return ops.cast_bf16(t, torch.empty(t.shape, device=t.device, dtype=BF16))


# ------------------------------------------------------------------------ fbank
@torch.library.custom_op("ste::fbank", mutates_args=())
def fbank(wav: Tensor, lengths: Tensor, t_max: int, pad_value: float = 1.0, mask_mode: int = 0) -> tuple[Tensor, Tensor]:
    return ops.fbank(wav.float().contiguous(), lengths.to(torch.int32).contiguous(), int(t_max), pad_value=pad_value,
                     mask_mode=mask_mode)


@fbank.register_fake
def _fbank_fake(wav, lengths, t_max, pad_value=1.0, mask_mode=0):
    return wav.new_empty(wav.shape[0], t_max, 160, dtype=F32), wav.new_empty(wav.shape[0], t_max, dtype=torch.int64)


# ----------------------------------------------------------------------- linear
@torch.library.custom_op("ste::linear", mutates_args=())
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None) -> Tensor:
    x2 = x.reshape(-1, x.shape[-1])
    y = ops.linear(_bf16(x2), _bf16(weight), None if bias is None else bias.float().contiguous())
    return y.view(*x.shape[:-1], weight.shape[0])


@linear.register_fake
def _linear_fake(x, weight, bias=None):
    return x.new_empty(*x.shape[:-1], weight.shape[0], dtype=F32)


def _linear_setup(ctx, inputs, output):
    x, weight, bias = inputs
    ctx.save_for_backward(x, weight)
    ctx.has_bias = bias is not None
    ctx.dtypes = (x.dtype, weight.dtype, None if bias is None else bias.dtype)


def _linear_bwd(ctx, dy):
    x, weight = ctx.saved_tensors
    N, K = weight.shape
    dy2 = _bf16(dy.reshape(-1, N).float())
    dx = ops.linear_dx(dy2, _bf16(weight)).view(*x.shape[:-1], K)
    dw = ops.linear_dw(dy2, _bf16(x.reshape(-1, K)))
    db = None
    if ctx.has_bias:
        db = ops.colsum(dy.reshape(-1, N).float().contiguous(), torch.zeros(N, device=dy.device, dtype=F32))
    xd, wd, bd = ctx.dtypes
    return dx.to(xd), dw.to(wd), (db.to(bd) if db is not None else None)


torch.library.register_autograd("ste::linear", _linear_bwd, setup_context=_linear_setup)


# ------------------------------------------------------------------- layer norm
@torch.library.custom_op("ste::layer_norm", mutates_args=())
def layer_norm(x: Tensor, weight: Tensor, bias: Tensor, eps: float = 1e-5) -> tuple[Tensor, Tensor, Tensor]:
    x2 = x.float().reshape(-1, x.shape[-1]).contiguous()
    y = torch.empty_like(x2)
    mean, rstd = ops.layernorm_fwd(x2, weight.float().contiguous(), bias.float().contiguous(), eps, y=y)
    return y.view(x.shape), mean, rstd


@layer_norm.register_fake
def _layer_norm_fake(x, weight, bias, eps=1e-5):
    rows = x.numel() // x.shape[-1]
    return x.new_empty(x.shape, dtype=F32), x.new_empty(rows, dtype=F32), x.new_empty(rows, dtype=F32)


def _ln_setup(ctx, inputs, output):
    x, weight, bias, eps = inputs
    ctx.save_for_backward(x, weight, bias, output[1], output[2])


def _ln_bwd(ctx, dy, _dmean, _drstd):
    x, weight, bias, mean, rstd = ctx.saved_tensors
    C = x.shape[-1]
    x2 = x.float().reshape(-1, C).contiguous()
    dx = torch.empty_like(x2)
    dg = torch.zeros(C, device=x.device, dtype=F32)
    db = torch.zeros(C, device=x.device, dtype=F32)
    ops.layernorm_bwd(dy.float().reshape(-1, C).contiguous(), x2, mean, rstd, weight.float().contiguous(),
                      beta=bias.float().contiguous(), dx=dx, dgamma=dg, dbeta=db)
    return dx.view(x.shape).to(x.dtype), dg.to(weight.dtype), db.to(bias.dtype), None


torch.library.register_autograd("ste::layer_norm", _ln_bwd, setup_context=_ln_setup)


# -------------------------------------------------------------------- attention
@torch.library.custom_op("ste::attention", mutates_args=())
def attention(q: Tensor, k: Tensor, v: Tensor, key_mask: Optional[Tensor], rel_E: Optional[Tensor], scale: float,
              rel_left: int = 64, rel_right: int = 8) -> tuple[Tensor, Tensor, Tensor]:
    """q/k/v [B, T, H*64] (bf16 or fp32), key_mask [B, T] (nonzero = valid) or None, rel_E
    [rel_left + rel_right + 1, 64] or None -> (o bf16 [B, T, H*64], lse fp32 [B*H*T], o_lo bf16)."""
    B, T, W = q.shape
    H = W // 64
    qb, kb, vb = (_bf16(t.reshape(B * T, W)) for t in (q, k, v))
    o = torch.empty(B * T, W, device=q.device, dtype=BF16)
    o_lo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=q.device, dtype=F32)
    km = None if key_mask is None else key_mask.to(torch.int32).reshape(-1).contiguous()
    E = None if rel_E is None else _bf16(rel_E)
    ops.attention_fwd(qb, kb, vb, B=B, T=T, H=H, o=o, lse=lse, key_mask=km, rel_E=E, rel_left=rel_left,
                      rel_right=rel_right, scale=scale, o_lo=o_lo)
    return o.view(B, T, W), lse, o_lo.view(B, T, W)


@attention.register_fake
def _attention_fake(q, k, v, key_mask, rel_E, scale, rel_left=64, rel_right=8):
    B, T, W = q.shape
    return (q.new_empty(B, T, W, dtype=BF16), q.new_empty(B * (W // 64) * T, dtype=F32),
            q.new_empty(B, T, W, dtype=BF16))


def _attn_setup(ctx, inputs, output):
    q, k, v, key_mask, rel_E, scale, rel_left, rel_right = inputs
    o, lse, o_lo = output
    ctx.save_for_backward(q, k, v, key_mask, rel_E, o, lse, o_lo)
    ctx.args = (scale, rel_left, rel_right)


def _attn_bwd(ctx, do, _dlse, _dolo):
    q, k, v, key_mask, rel_E, o, lse, o_lo = ctx.saved_tensors
    scale, rel_left, rel_right = ctx.args
    B, T, W = q.shape
    H = W // 64
    qb, kb, vb = (_bf16(t.reshape(B * T, W)) for t in (q, k, v))
    dq, dk, dv = (torch.empty(B * T, W, device=q.device, dtype=BF16) for _ in range(3))
    delta = torch.empty(B * H * T, device=q.device, dtype=F32)
    km = None if key_mask is None else key_mask.to(torch.int32).reshape(-1).contiguous()
    E = None if rel_E is None else _bf16(rel_E)
    dE = None if rel_E is None else torch.zeros(rel_E.shape, device=q.device, dtype=F32)
    gwork = None if rel_E is None else torch.empty(B * H * T * 80, device=q.device, dtype=F32)
    ops.attention_bwd(qb, kb, vb, o.reshape(B * T, W), lse, _bf16(do.reshape(B * T, W)), dq, dk, dv, B=B, T=T, H=H,
                      delta=delta, key_mask=km, rel_E=E, rel_left=rel_left, rel_right=rel_right, scale=scale, dE=dE,
                      gwork=gwork, o_lo=o_lo.reshape(B * T, W))
    return (dq.view(B, T, W).to(q.dtype), dk.view(B, T, W).to(k.dtype), dv.view(B, T, W).to(v.dtype), None,
            None if dE is None else dE.to(rel_E.dtype), None, None, None)


torch.library.register_autograd("ste::attention", _attn_bwd, setup_context=_attn_setup)


# -------------------------------------------------------------------- pair loss
@torch.library.custom_op("ste::pair_loss", mutates_args=())
def pair_loss(s_pos: Tensor, s_neg: Tensor, alignment_scores: Optional[Tensor], temperature: float = 0.1,
              alignment_weight: float = 0.3, corrupt_gamma: float = 0.35) -> Tensor:
    B = s_pos.shape[0]
    flat = torch.cat([s_pos.float(), s_neg.float()]).contiguous()
    sp, sn = torch.empty(B, device=s_pos.device), torch.empty(B, device=s_pos.device)
    loss = torch.empty(1, device=s_pos.device)
    al = None if alignment_scores is None else alignment_scores.float().contiguous()
    L = 0 if al is None else al.shape[1]
    # ste_pair_loss_fwd reads S[i*ldS + i] / S[i*ldS + off_neg + i]: ldS = 0 makes that flat[i] / flat[B + i]
    _lib.call("ste_pair_loss_fwd", flat.data_ptr(), 0, B, None if al is None else al.data_ptr(), B, L,
              float(temperature), float(alignment_weight), float(corrupt_gamma), sp.data_ptr(), sn.data_ptr(),
              loss.data_ptr(), _lib.stream_ptr())
    return loss.reshape(())


@pair_loss.register_fake
def _pair_loss_fake(s_pos, s_neg, alignment_scores, temperature=0.1, alignment_weight=0.3, corrupt_gamma=0.35):
    return s_pos.new_empty((), dtype=F32)


def _pl_setup(ctx, inputs, output):
    s_pos, s_neg, al, temperature, aw, gamma = inputs
    ctx.save_for_backward(s_pos, s_neg, al)
    ctx.args = (temperature, aw, gamma)


def _pl_bwd(ctx, dloss):
    s_pos, s_neg, al = ctx.saved_tensors
    tau, aw, gamma = ctx.args
    B = s_pos.shape[0]
    dsp, dsn = torch.empty(B, device=s_pos.device), torch.empty(B, device=s_pos.device)
    alf = None if al is None else al.float().contiguous()
    L = 0 if alf is None else alf.shape[1]
    dal = None if alf is None else torch.empty(B, L, device=s_pos.device)
    ops.pair_loss_bwd(s_pos.float().contiguous(), s_neg.float().contiguous(), alf, B, L, tau, aw, gamma,
                      dloss.reshape(1).float().contiguous(), dsp, dsn, dal)
    return (dsp.to(s_pos.dtype), dsn.to(s_neg.dtype), None if dal is None else dal.to(al.dtype), None, None, None)


torch.library.register_autograd("ste::pair_loss", _pl_bwd, setup_context=_pl_setup)


# ------------------------------------------------------------------------ AdamW
@torch.library.custom_op("ste::adamw_", mutates_args=("p", "m", "v", "p_bf16"))
def adamw_(p: Tensor, g: Tensor, m: Tensor, v: Tensor, p_bf16: Tensor, lr: float, beta1: float, beta2: float,
           eps: float, weight_decay: float, step: int, sumsq: Optional[Tensor] = None, max_norm: float = 1.0) -> None:
    """One AdamW step (torch.optim.AdamW semantics, decoupled decay) on flat fp32 p/g/m/v; g is
    scaled by clip_grad_norm_'s min(1, max_norm/(sqrt(sumsq)+1e-6)) when sumsq (fp64 Σg²) is given;
    p_bf16 receives the bf16 copy of the new p."""
    ops.adamw(p, g, m, v, p_bf16, lr=lr, beta1=beta1, beta2=beta2, eps=eps, wd=weight_decay, step=step,
              sumsq_acc=sumsq, max_norm=max_norm)


@adamw_.register_fake
def _adamw_fake(p, g, m, v, p_bf16, lr, beta1, beta2, eps, weight_decay, step, sumsq=None, max_norm=1.0):
    return None


OPS = ("fbank", "linear", "layer_norm", "attention", "pair_loss", "adamw_")
