"""Thin typed wrappers over the libste.so C ABI (include/ste.h).

Each function takes torch tensors that already live on the GPU, builds the C
argument block and launches on the current HIP stream.  No function allocates
hidden state or falls back to torch math: a bad shape returns a non-zero status
from the library and surfaces as SteError.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import GemmArgs, LnFwdArgs, LnBwdArgs, AttnArgs, ptr, call

BF16 = torch.bfloat16
F32 = torch.float32


def _s():
    return _lib.stream_ptr()


def _ld(t: torch.Tensor) -> int:
    assert t.dim() >= 2 and t.stride(-1) == 1, "row-major operand required"
    return t.stride(-2)


# ------------------------------------------------------------------- GEMM
def gemm(a, b, *, a_kc=True, b_kc=True, M=None, N=None, K=None, out=None, out_bf16=False, bias=None,
         act=_lib.ACT_NONE, pre_out=None, z=None, residual=None, alpha=1.0, beta=0.0, colsum=None,
         row_scale=None, drop_p=0.0, seed=0, out_bf16_copy=None, batch=1, stride_a=0, stride_b=0, stride_c=0,
         stride_r=0, drop_ld=0):
    """out[M,N] = epilogue(alpha * A·B).  See include/ste.h for the epilogue order.

    a_kc: A is [M,K] row-major (else [K,M]);  b_kc: B is [N,K] row-major (else [K,N]).
    """
    assert a.dtype == BF16 and b.dtype == BF16, "GEMM operands are bf16"
    if M is None:
        M = a.shape[-2] if a_kc else a.shape[-1]
    if K is None:
        K = a.shape[-1] if a_kc else a.shape[-2]
    if N is None:
        N = b.shape[-2] if b_kc else b.shape[-1]
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=BF16 if out_bf16 else F32)
    args = GemmArgs()
    args.M, args.N, args.K, args.batch = M, N, K, batch
    args.A, args.lda, args.a_kc = ptr(a), _ld(a), int(a_kc)
    args.B, args.ldb, args.b_kc = ptr(b), _ld(b), int(b_kc)
    args.strideA, args.strideB, args.strideC, args.strideR = stride_a, stride_b, stride_c, stride_r
    args.C, args.ldc, args.c_bf16 = ptr(out), _ld(out), int(out.dtype == BF16)
    if pre_out is not None:
        args.C2, args.ldc2 = ptr(pre_out), _ld(pre_out)
    if out_bf16_copy is not None:
        args.C3, args.ldc3 = ptr(out_bf16_copy), _ld(out_bf16_copy)
    if bias is not None:
        assert bias.dtype == F32 and bias.is_contiguous()
        args.bias = ptr(bias)
    if residual is not None:
        args.R, args.ldr, args.r_bf16 = ptr(residual), _ld(residual), int(residual.dtype == BF16)
    if z is not None:
        args.Z, args.ldz = ptr(z), _ld(z)
    if colsum is not None:
        assert colsum.dtype == F32
        args.colsum = ptr(colsum)
    if row_scale is not None:
        args.row_scale = ptr(row_scale)
    args.alpha, args.beta, args.act = float(alpha), float(beta), int(act)
    args.drop_p, args.seed, args.drop_ld = float(drop_p), int(seed) & (2**64 - 1), int(drop_ld)
    call("ste_gemm", C.byref(args), _s())
    return out


def linear(x, w, bias=None, **kw):
    """y = x·wᵀ (+bias) with x [M,K] bf16, w [N,K] bf16 (nn.Linear layout)."""
    return gemm(x, w, a_kc=True, b_kc=True, bias=bias, **kw)


def linear_dx(dy, w, **kw):
    """dx = dy·w with dy [M,N] bf16, w [N,K] bf16 -> [M,K]."""
    return gemm(dy, w, a_kc=True, b_kc=False, M=dy.shape[0], N=w.shape[1], K=dy.shape[1], **kw)


def linear_dw(dy, x, **kw):
    """dw = dyᵀ·x with dy [M,N] bf16, x [M,K] bf16 -> [N,K]."""
    return gemm(dy, x, a_kc=False, b_kc=False, M=dy.shape[1], N=x.shape[1], K=dy.shape[0], **kw)


# -------------------------------------------------------------- LayerNorm
def layernorm_fwd(x, gamma, beta, eps, *, y=None, yb=None, mean=None, rstd=None, row_scale=None,
                  act=_lib.ACT_NONE, drop_p=0.0, seed=0):
    rows, cols = x.shape
    if mean is None:
        mean = torch.empty(rows, device=x.device, dtype=F32)
    if rstd is None:
        rstd = torch.empty(rows, device=x.device, dtype=F32)
    a = LnFwdArgs()
    a.rows, a.cols = rows, cols
    a.x, a.ldx, a.x_bf16 = ptr(x), _ld(x), int(x.dtype == BF16)
    a.gamma, a.beta, a.eps = ptr(gamma), ptr(beta), float(eps)
    if y is not None:
        a.y, a.ldy = ptr(y), _ld(y)
    if yb is not None:
        a.yb, a.ldyb = ptr(yb), _ld(yb)
    a.mean, a.rstd = ptr(mean), ptr(rstd)
    a.row_scale = ptr(row_scale)
    a.act, a.drop_p, a.seed = int(act), float(drop_p), int(seed) & (2**64 - 1)
    call("ste_layernorm_fwd", C.byref(a), _s())
    return mean, rstd


def layernorm_bwd(dy, x, mean, rstd, gamma, *, beta=None, dx=None, dxb=None, dres=None, dgamma=None, dbeta=None,
                  row_scale=None, act=_lib.ACT_NONE, drop_p=0.0, seed=0, out_scale=1.0, in_drop_p=0.0, in_seed=0):
    rows, cols = x.shape
    a = LnBwdArgs()
    a.rows, a.cols = rows, cols
    a.dy, a.lddy, a.dy_bf16 = ptr(dy), _ld(dy), int(dy.dtype == BF16)
    a.x, a.ldx, a.x_bf16 = ptr(x), _ld(x), int(x.dtype == BF16)
    a.mean, a.rstd, a.gamma, a.beta = ptr(mean), ptr(rstd), ptr(gamma), ptr(beta)
    a.row_scale, a.act = ptr(row_scale), int(act)
    if dres is not None:
        a.dres, a.lddres = ptr(dres), _ld(dres)
    if dx is not None:
        a.dx, a.lddx = ptr(dx), _ld(dx)
    if dxb is not None:
        a.dxb, a.lddxb = ptr(dxb), _ld(dxb)
    a.dgamma, a.dbeta = ptr(dgamma), ptr(dbeta)
    a.drop_p, a.seed, a.out_scale = float(drop_p), int(seed) & (2**64 - 1), float(out_scale)
    a.in_drop_p, a.in_seed = float(in_drop_p), int(in_seed) & (2**64 - 1)
    call("ste_layernorm_bwd", C.byref(a), _s())
    return dx, dxb
