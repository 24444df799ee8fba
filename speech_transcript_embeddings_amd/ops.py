"""Thin typed wrappers over the libste.so C ABI (include/ste.h).

Each function takes torch tensors that already live on the GPU, builds the C
argument block and launches on the current HIP stream.  No function allocates
hidden state or falls back to torch math: a bad shape returns a non-zero status
from the library and surfaces as SteError.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib
from ._lib import GemmArgs, LnFwdArgs, LnBwdArgs, AttnArgs, ptr, call, fn

BF16 = torch.bfloat16
F32 = torch.float32


def _s():
    return _lib.stream_ptr()


def _ld(t: torch.Tensor) -> int:
    assert t.dim() >= 2 and t.stride(-1) == 1, "row-major operand required"
    return t.stride(-2)


# True: column / table-row reductions through the library's fp32 atomics (its workspace-free path;
# A/B runs and tests; STE_ATOMIC_SUMS=1 sets it for a whole run under the A/B build).  Default: ordered partial sums,
# run-to-run deterministic gradients.
ATOMIC_SUMS = _lib.ab_env("STE_ATOMIC_SUMS", "0") == "1"
_RED_WS = {}


def _red_ws(dev, floats):
    """Partial-sum workspace of the current stream for the ordered reductions (GEMM bias gradients,
    ste_colsum, depthwise-conv / embedding / SpecAugment gradients), grown on demand.  Launches of
    one stream run in order, so consecutive reductions reuse it; concurrent streams get their own.
    None under ATOMIC_SUMS."""
    if ATOMIC_SUMS or floats <= 0:
        return None
    key = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
    w = _RED_WS.get(key)
    if w is None or w.numel() < floats:
        w = _RED_WS[key] = torch.empty(max(int(floats), 1 << 20), device=dev, dtype=F32)
    return w


def _ws_args(w):
    return (None, 0) if w is None else (ptr(w), w.numel())


# ------------------------------------------------------------------- GEMM
def gemm(a, b, *, a_kc=True, b_kc=True, M=None, N=None, K=None, out=None, out_bf16=False, bias=None,
         act=_lib.ACT_NONE, pre_out=None, z=None, residual=None, alpha=1.0, beta=0.0, colsum=None,
         row_scale=None, drop_p=0.0, seed=0, out_bf16_copy=None, batch=1, stride_a=0, stride_b=0, stride_c=0,
         stride_r=0, drop_ld=0, ws=None, mx8=None, copy_lo=False):
    """out[M,N] = epilogue(alpha * A·B).  See include/ste.h for the epilogue order.

    a_kc: A is [M,K] row-major (else [K,M]);  b_kc: B is [N,K] row-major (else [K,N]).
    bf16 operands run on ste_gemm; fp32 operands (pre_out / z fp32 too) on ste_gemm_f32, the
    exact-f32 matrix-core GEMM of the heads.
    """
    f32 = mx8 is None and a.dtype == F32
    if mx8 is not None:  # (a_scales, b_scales): e4m3 operands with E8M0 block scales (ste_gemm_mx8)
        assert a.dtype == torch.uint8 and b.dtype == torch.uint8 and a_kc and b_kc, "MX-fp8 GEMM operands"
    elif f32:
        assert b.dtype == F32 and batch == 1, "ste_gemm_f32: fp32 operands, batch 1"
        assert (pre_out is None or pre_out.dtype == F32) and (z is None or z.dtype == F32)
    else:
        assert a.dtype == BF16 and b.dtype == BF16, "GEMM operands are bf16 (or both fp32)"
    if M is None:
        M = a.shape[-2] if a_kc else a.shape[-1]
    if K is None:
        K = a.shape[-1] if a_kc else a.shape[-2]
    if N is None:
        N = b.shape[-2] if b_kc else b.shape[-1]
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=BF16 if out_bf16 else F32)
    elif out is False:
        assert mx8 is not None and len(mx8) > 2, "out=False: MX-fp8 GEMM with an fp8 output only"
    args = GemmArgs()
    args.M, args.N, args.K, args.batch = M, N, K, batch
    args.A, args.lda, args.a_kc = ptr(a), _ld(a), int(a_kc)
    args.B, args.ldb, args.b_kc = ptr(b), _ld(b), int(b_kc)
    args.strideA, args.strideB, args.strideC, args.strideR = stride_a, stride_b, stride_c, stride_r
    if out is not False:
        args.C, args.ldc, args.c_bf16 = ptr(out), _ld(out), int(out.dtype == BF16)
    else:
        args.ldc, args.c_bf16 = N, int(out_bf16)
    if pre_out is not None:
        args.C2, args.ldc2 = ptr(pre_out), _ld(pre_out)
    if out_bf16_copy is not None:   # copy_lo: it receives bf16(v - bf16(v)) (a [hi | lo] split output)
        args.C3, args.ldc3, args.c3_lo = ptr(out_bf16_copy), _ld(out_bf16_copy), int(bool(copy_lo))
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
    if colsum is not None and mx8 is None and not ATOMIC_SUMS:
        # deterministic bias gradients: the ordered partial-sum plan needs a workspace this large
        need = int(fn("ste_gemm_colsum_ws_floats")(C.byref(args)))
        if ws is None or ws.numel() < need:
            ws = _red_ws(a.device, need)
    if ws is not None:  # split-K workspace (weight gradients) / column-sum partials, see include/ste.h
        assert ws.dtype == F32 and ws.is_contiguous()
        args.ws, args.ws_bytes = ptr(ws), ws.numel() * 4
    if mx8 is not None:
        q8 = mx8[2] if len(mx8) > 2 else (None, None)
        if out is False:  # fp8 copy only
            args.C = None

        def launch():
            call("ste_gemm_mx8", C.byref(args), ptr(mx8[0]), ptr(mx8[1]), ptr(q8[0]), ptr(q8[1]), _s())
        # which MX kernel the library plans (the persistent 8-phase one or the single-stage one)
        name = "gemm_mx8_kernel" if GEMM_TRACE is None or not int(fn("ste_gemm_mx8_kernel")(
            C.byref(args), int(q8[0] is not None))) else "gemm_8ph_kernel<mx8>"
    elif f32:
        def launch():
            call("ste_gemm_f32", C.byref(args), _s())
        name = "gemm_f32_kernel"
    else:
        def launch():
            call("ste_gemm", C.byref(args), _s())
        name = None
    if GEMM_CENSUS is not None and name is None:
        key = "%s act=%d M=%d N=%d K=%d batch=%d %s" % (
            gemm_kernel_name(args), act, M, N, K, batch,
            "".join(f for f, v in (("B", bias), ("C2", pre_out), ("Z", z), ("R", residual), ("CS", colsum),
                                   ("RS", row_scale), ("C3", out_bf16_copy)) if v is not None)
            + ("D" if drop_p > 0 else "") + ("beta" if beta != 0 else "") + ("bf16" if out_bf16 or (
                out is not None and out is not False and out.dtype == BF16) else ""))
        GEMM_CENSUS[key] = GEMM_CENSUS.get(key, 0) + 1
    if GEMM_TRACE is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        launch()
        ev1.record()
        GEMM_TRACE.append((name or gemm_kernel_name(args), 2.0 * M * N * K * batch, ev0, ev1, (M, N, K, batch),
                           torch.cuda.current_stream().cuda_stream))
    else:
        launch()
    return q8 if out is False else out


GEMM_TRACE = None  # list while bench.py measures per-launch GEMM durations with HIP events
# STE_GEMM_CENSUS=<file>: count bf16 GEMM launches per (kernel, epilogue features, shape) and
# write the table at exit (profiles/ tooling: which launches miss a compiled epilogue)
GEMM_CENSUS = {} if os.environ.get("STE_GEMM_CENSUS") else None
if GEMM_CENSUS is not None:
    import atexit
    import json

    atexit.register(lambda: open(os.environ["STE_GEMM_CENSUS"], "w").write(
        json.dumps(dict(sorted(GEMM_CENSUS.items())), indent=1)))
# list while bench.py measures the HBM-bound kernels (fbank, LayerNorm): (name, algorithmic
# bytes, ev0, ev1) per launch, timed with HIP events on the launching (current) stream
HBM_TRACE = None


def _traced(name, nbytes, launch):
    if HBM_TRACE is None:
        launch()
        return
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    launch()
    ev1.record()
    HBM_TRACE.append((name, float(nbytes), ev0, ev1, torch.cuda.current_stream().cuda_stream))


def _nb(t):
    return 0 if t is None else t.numel() * t.element_size()


def gemm_kernel_name(args: GemmArgs) -> str:
    """The kernel symbol rocprofv3 reports for this launch (asks the library which one it picks)."""
    buf = C.create_string_buffer(128)
    call("ste_gemm_kernel_name", C.byref(args), buf, 128)
    return buf.value.decode()


def gemm_plan_min_tiles(bf16=0, mx8=0):
    """Set the 8-phase kernels' plan thresholds (ste_gemm_plan_min_tiles: fewest 256x256 output
    tiles; <= 0 keeps one) and return the previous (bf16, mx8) pair."""
    pb, pm = C.c_int(), C.c_int()
    call("ste_gemm_plan_min_tiles", int(bf16), int(mx8), C.byref(pb), C.byref(pm))
    return pb.value, pm.value


class bench_gemm_plan:
    """Context manager for parity tests: every GEMM with at least one 256x256 output tile is planned
    on the persistent 8-phase kernels (bf16 and MX-fp8) the b = 64 bench step runs, so a B <= 4
    batch exercises the same compile-time epilogue instantiations (their guarded partial-tile path
    at the edges); the library's thresholds are restored on exit."""

    def __enter__(self):
        self.prev = gemm_plan_min_tiles(1, 1)
        return self

    def __exit__(self, *exc):
        gemm_plan_min_tiles(*self.prev)


def linear(x, w, bias=None, **kw):
    """y = x·wᵀ (+bias) with x [M,K] bf16, w [N,K] bf16 (nn.Linear layout)."""
    return gemm(x, w, a_kc=True, b_kc=True, bias=bias, **kw)


def mx8_quant(x, q=None, scales=None):
    """bf16 [rows, K] -> (e4m3 bytes [rows, K], E8M0 scales [rows, K/32]) (ste_mx8_quant)."""
    rows, K = x.shape
    if q is None:
        q = torch.empty((rows, K), device=x.device, dtype=torch.uint8)
    if scales is None:
        scales = torch.empty((rows, K // 32), device=x.device, dtype=torch.uint8)
    call("ste_mx8_quant", ptr(x), _ld(x), rows, K, ptr(q), ptr(scales), _s())
    return q, scales


def linear_mx8(xq, wq, bias=None, q_out=None, **kw):
    """y = x·wᵀ (+bias) on the MX-fp8 GEMM: xq = (e4m3 [M,K], scales), wq = (e4m3 [N,K], scales).
    q_out = (e4m3 [M,N], scales [M,N/32]): also write y MX-fp8 quantised; with out=False only that."""
    mx8 = (xq[1], wq[1]) if q_out is None else (xq[1], wq[1], q_out)
    return gemm(xq[0], wq[0], a_kc=True, b_kc=True, bias=bias, mx8=mx8, **kw)


def linear_dx(dy, w, **kw):
    """dx = dy·w with dy [M,N] bf16, w [N,K] bf16 -> [M,K]."""
    return gemm(dy, w, a_kc=True, b_kc=False, M=dy.shape[0], N=w.shape[1], K=dy.shape[1], **kw)


def linear_dw(dy, x, **kw):
    """dw = dyᵀ·x with dy [M,N] bf16, x [M,K] bf16 -> [N,K]."""
    return gemm(dy, x, a_kc=False, b_kc=False, M=dy.shape[1], N=x.shape[1], K=dy.shape[0], **kw)


# -------------------------------------------------------------- LayerNorm
_LN_WS = {}


def _ln_ws_floats(rows, cols):
    """ste_layernorm_bwd_ws_floats (cached per shape)."""
    n = _LN_WS.get((rows, cols))
    if n is None:
        n = _LN_WS[(rows, cols)] = int(_lib.fn("ste_layernorm_bwd_ws_floats")(rows, cols))
    return n


def _ln_fwd_struct(x, gamma, beta, eps, y=None, yb=None, mean=None, rstd=None, row_scale=None, act=_lib.ACT_NONE,
                   drop_p=0.0, seed=0, q8=None, rows=None, cols=None, ylo=None):
    """-> (LnFwdArgs, mean, rstd, algorithmic bytes).  x may be None (pair kernels: the second
    LN's input is the first one's output in registers); then rows/cols are given."""
    if x is not None:
        rows, cols = x.shape
    dev = gamma.device
    if mean is None:
        mean = torch.empty(rows, device=dev, dtype=F32)
    if rstd is None:
        rstd = torch.empty(rows, device=dev, dtype=F32)
    a = LnFwdArgs()
    a.rows, a.cols = rows, cols
    if x is not None:
        a.x, a.ldx, a.x_bf16 = ptr(x), _ld(x), int(x.dtype == BF16)
    a.gamma, a.beta, a.eps = ptr(gamma), ptr(beta), float(eps)
    if y is not None:
        a.y, a.ldy = ptr(y), _ld(y)
    if yb is not None:
        a.yb, a.ldyb = ptr(yb), _ld(yb)
    if ylo is not None:   # the low half bf16(y - bf16(y)): with yb, a [hi | lo] split image
        assert yb is not None
        a.ylo, a.ldylo = ptr(ylo), _ld(ylo)
    a.mean, a.rstd = ptr(mean), ptr(rstd)
    a.row_scale = ptr(row_scale)
    a.act, a.drop_p, a.seed = int(act), float(drop_p), int(seed) & (2**64 - 1)
    if q8 is not None:  # (e4m3 [rows, cols], E8M0 [rows, cols/32]): MX-fp8 copy for ste_gemm_mx8
        a.q8, a.q8s, a.ldq8 = ptr(q8[0]), ptr(q8[1]), _ld(q8[0])
    # algorithmic bytes: read x, write every requested output, 8 B/row of statistics
    nbytes = rows * cols * ((x.element_size() if x is not None else 0) + (4 if y is not None else 0) +
                            (2 if yb is not None else 0) + (2 if ylo is not None else 0) +
                            (1 + 1 / 32 if q8 is not None else 0)) + 8 * rows + 8 * cols
    return a, mean, rstd, nbytes


def layernorm_fwd(x, gamma, beta, eps, *, y=None, yb=None, mean=None, rstd=None, row_scale=None,
                  act=_lib.ACT_NONE, drop_p=0.0, seed=0, q8=None, ylo=None):
    a, mean, rstd, nbytes = _ln_fwd_struct(x, gamma, beta, eps, y, yb, mean, rstd, row_scale, act, drop_p, seed, q8,
                                           ylo=ylo)
    _traced("layernorm_fwd", nbytes, lambda: call("ste_layernorm_fwd", C.byref(a), _s()))
    return mean, rstd


def layernorm_fwd_pair(first: dict, second: dict):
    """y2 = LN_2(LN_1(x)) in one pass (ste_layernorm_fwd_pair): `first` / `second` are
    layernorm_fwd keyword sets (x, gamma, beta, eps, y/yb/q8 ...); `second` has no x.  Returns
    ((mean1, rstd1), (mean2, rstd2))."""
    a, m1, r1, nb1 = _ln_fwd_struct(**first)
    b, m2, r2, nb2 = _ln_fwd_struct(None, rows=a.rows, cols=a.cols, **second)
    _traced("layernorm_fwd_pair", nb1 + nb2, lambda: call("ste_layernorm_fwd_pair", C.byref(a), C.byref(b), _s()))
    return (m1, r1), (m2, r2)


# True: LayerNorm column sums through fp32 atomics (the library's workspace-free path; A/B and tests;
# STE_LN_ATOMIC=1 sets it for a whole run under the A/B build)
LN_ATOMIC_COLSUMS = _lib.ab_env("STE_LN_ATOMIC", "0") == "1"


_LN_WS_BUF = {}


def _ln_ws(dev, rows, cols, slot):
    """Column-partial workspace of a LayerNorm backward, one per (stream, slot), grown on demand:
    the launches of one stream run in order, so consecutive backwards reuse one buffer (a pair
    kernel's two LayerNorms take slots 0 and 1); concurrent streams get their own.  Its size
    (ste_layernorm_bwd_ws_floats) stops growing once rows reach the kernel's block count, so
    batches padded to different lengths share one buffer instead of one each."""
    key = (torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0, slot)
    need = _ln_ws_floats(rows, cols)
    w = _LN_WS_BUF.get(key)
    if w is None or w.numel() < need:
        w = _LN_WS_BUF[key] = torch.empty(need, device=dev, dtype=F32)
    return w


def _ln_bwd_struct(dy, x, mean, rstd, gamma, beta=None, dx=None, dxb=None, dres=None, dgamma=None, dbeta=None,
                   row_scale=None, act=_lib.ACT_NONE, drop_p=0.0, seed=0, out_scale=1.0, in_drop_p=0.0, in_seed=0,
                   out_row_scale=None, dsum=None, _slot=0):
    """-> (LnBwdArgs, algorithmic bytes).  dy may be None (the first LN of a backward pair
    takes its gradient from the second one's, in registers)."""
    rows, cols = x.shape
    a = LnBwdArgs()
    a.rows, a.cols = rows, cols
    if dy is not None:
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
    a.out_row_scale, a.dsum = ptr(out_row_scale), ptr(dsum)
    ws = None
    if (dgamma is not None or dbeta is not None or dsum is not None) and not LN_ATOMIC_COLSUMS:
        # per-block column partials, summed in a fixed order by the library (deterministic)
        ws = _ln_ws(x.device, rows, cols, _slot)
        a.ws, a.ws_floats = ptr(ws), ws.numel()
    # algorithmic bytes: read dy, x (and dres), write dx / dxb, 8 B/row of statistics
    nbytes = rows * cols * ((dy.element_size() if dy is not None else 0) + x.element_size() +
                            (4 if dres is not None else 0) + (4 if dx is not None else 0) +
                            (2 if dxb is not None else 0)) + 8 * rows + 16 * cols
    return a, nbytes, ws


def layernorm_bwd(dy, x, mean, rstd, gamma, *, beta=None, dx=None, dxb=None, dres=None, dgamma=None, dbeta=None,
                  row_scale=None, act=_lib.ACT_NONE, drop_p=0.0, seed=0, out_scale=1.0, in_drop_p=0.0, in_seed=0,
                  out_row_scale=None, dsum=None):
    a, nbytes, _ws = _ln_bwd_struct(dy, x, mean, rstd, gamma, beta, dx, dxb, dres, dgamma, dbeta, row_scale, act,
                                    drop_p, seed, out_scale, in_drop_p, in_seed, out_row_scale, dsum)
    _traced("layernorm_bwd", nbytes, lambda: call("ste_layernorm_bwd", C.byref(a), _s()))
    return dx, dxb


def layernorm_bwd_pair(first: dict, second: dict):
    """Backward of layernorm_fwd_pair in one pass (ste_layernorm_bwd_pair): `second` (the later
    LN, with its dy) runs first and its input gradient feeds `first` in registers (`first` has
    no dy; second's dx output is optional).  Keyword sets as layernorm_bwd."""
    a, nb1, _wa = _ln_bwd_struct(None, **first, _slot=1)
    b, nb2, _wb = _ln_bwd_struct(**second)
    _traced("layernorm_bwd_pair", nb1 + nb2, lambda: call("ste_layernorm_bwd_pair", C.byref(a), C.byref(b), _s()))


# -------------------------------------------------------------- attention
def attention_fwd(q, k, v, *, B, T, H, o, lse, key_mask=None, rel_E=None, rel_left=64, rel_right=8,
                  scale=0.125, drop_p=0.0, seed=0, o_lo=None, zero_masked_rows=False):
    """q/k/v/o: bf16 [B*T, *] views (row-major, head h at columns h*64..), lse fp32 [B*H*T].
    o_lo (optional, bf16 like o): receives bf16(O - bf16(O)) for the backward's delta."""
    a = AttnArgs()
    a.B, a.T, a.H = B, T, H
    a.q, a.ldq = ptr(q), _ld(q)
    a.k, a.ldk = ptr(k), _ld(k)
    a.v, a.ldv = ptr(v), _ld(v)
    a.o, a.ldo = ptr(o), _ld(o)
    a.lse = ptr(lse)
    a.key_mask = ptr(key_mask)
    a.rel_E, a.rel_left, a.rel_right = ptr(rel_E), rel_left, rel_right
    a.scale, a.drop_p, a.seed = float(scale), float(drop_p), int(seed) & (2**64 - 1)
    if o_lo is not None:
        a.o_lo, a.ldolo = ptr(o_lo), _ld(o_lo)
    a.zero_masked_rows = int(bool(zero_masked_rows))
    call("ste_attention_fwd", C.byref(a), _s())
    return a


def attention_fwd_f32(q, k, v, *, B, T, H, o32, lse, o=None, o_lo=None, key_mask=None, scale=0.125, drop_p=0.0,
                      seed=0, zero_masked_rows=False):
    """fp32 q/k/v [B*T, *] views -> O fp32 (o32) + optional bf16 hi / lo copies for the bf16
    backward, lse fp32 [B*H*T] (ste_attention_fwd_f32: the text encoder's precise forward)."""
    assert q.dtype == F32 and k.dtype == F32 and v.dtype == F32 and (o32 is None or o32.dtype == F32)
    a = AttnArgs()
    a.B, a.T, a.H = B, T, H
    a.q, a.ldq = ptr(q), _ld(q)
    a.k, a.ldk = ptr(k), _ld(k)
    a.v, a.ldv = ptr(v), _ld(v)
    if o is not None:
        a.o, a.ldo = ptr(o), _ld(o)
    if o_lo is not None:
        a.o_lo, a.ldolo = ptr(o_lo), _ld(o_lo)
    a.lse = ptr(lse)
    a.key_mask = ptr(key_mask)
    a.scale, a.drop_p, a.seed = float(scale), float(drop_p), int(seed) & (2**64 - 1)
    a.zero_masked_rows = int(bool(zero_masked_rows))
    call("ste_attention_fwd_f32", C.byref(a), ptr(o32), 0 if o32 is None else _ld(o32), _s())


def attention_bwd_f32(q, k, v, o, o_lo, lse, dout, dq, dk, dv, *, B, T, H, key_mask=None, scale=0.125, drop_p=0.0,
                      seed=0, zero_masked_rows=False):
    """Backward of attention_fwd_f32 in fp32 (ste_attention_bwd_f32): q/k/v/dout fp32 [B*T, *] views,
    o / o_lo the forward's bf16 hi / lo halves of O, lse as it saved -> dq/dk/dv fp32 views."""
    for t in (q, k, v, dout, dq, dk, dv):
        assert t.dtype == F32
    assert o.dtype == BF16 and o_lo.dtype == BF16
    a = AttnArgs()
    a.B, a.T, a.H = B, T, H
    a.q, a.ldq = ptr(q), _ld(q)
    a.k, a.ldk = ptr(k), _ld(k)
    a.v, a.ldv = ptr(v), _ld(v)
    a.o, a.ldo = ptr(o), _ld(o)
    a.o_lo, a.ldolo = ptr(o_lo), _ld(o_lo)
    a.lse = ptr(lse)
    a.key_mask = ptr(key_mask)
    a.scale, a.drop_p, a.seed = float(scale), float(drop_p), int(seed) & (2**64 - 1)
    a.zero_masked_rows = int(bool(zero_masked_rows))
    a.dout, a.lddo = ptr(dout), _ld(dout)
    a.dq, a.lddq = ptr(dq), _ld(dq)
    a.dk, a.lddk = ptr(dk), _ld(dk)
    a.dv, a.lddv = ptr(dv), _ld(dv)
    call("ste_attention_bwd_f32", C.byref(a), _s())


def split_bf16(x, nblk, lo_mask, out=None):
    """fp32 [rows, K] -> bf16 [rows, nblk·K]: copy i = bf16(x), or its low half bf16(x - bf16(x)) where
    bit i of lo_mask is set (ste_split_bf16)."""
    rows, K = x.shape
    if out is None:
        out = torch.empty((rows, nblk * K), device=x.device, dtype=BF16)
    assert out.shape == (rows, nblk * K) and out.is_contiguous() and out.dtype == BF16
    call("ste_split_bf16", ptr(x), _ld(x), rows, K, ptr(out), int(nblk), int(lo_mask), _s())
    return out


def linear_x2(x, w2, bias=None, **kw):
    """y = x·w_bf16ᵀ (+bias) with x fp32 [M, K] kept to ~16 mantissa bits, on the bf16 MFMA: one
    GEMM over K' = 2K of [x_hi | x_lo]·[w | w]ᵀ (w2 = ParamStore.w2, the bf16 weight twice)."""
    return gemm(split_bf16(x, 2, 2), w2, a_kc=True, b_kc=True, bias=bias, **kw)


def attention_bwd(q, k, v, o, lse, dout, dq, dk, dv, *, B, T, H, delta, key_mask=None, rel_E=None, rel_left=64,
                  rel_right=8, scale=0.125, drop_p=0.0, seed=0, dE=None, gwork=None, o_lo=None):
    a = AttnArgs()
    a.B, a.T, a.H = B, T, H
    a.q, a.ldq = ptr(q), _ld(q)
    a.k, a.ldk = ptr(k), _ld(k)
    a.v, a.ldv = ptr(v), _ld(v)
    a.o, a.ldo = ptr(o), _ld(o)
    a.lse = ptr(lse)
    a.key_mask = ptr(key_mask)
    a.rel_E, a.rel_left, a.rel_right = ptr(rel_E), rel_left, rel_right
    a.scale, a.drop_p, a.seed = float(scale), float(drop_p), int(seed) & (2**64 - 1)
    a.dout, a.lddo = ptr(dout), _ld(dout)
    a.dq, a.lddq = ptr(dq), _ld(dq)
    a.dk, a.lddk = ptr(dk), _ld(dk)
    a.dv, a.lddv = ptr(dv), _ld(dv)
    a.delta, a.dE, a.gwork = ptr(delta), ptr(dE), ptr(gwork)
    if o_lo is not None:
        a.o_lo, a.ldolo = ptr(o_lo), _ld(o_lo)
    call("ste_attention_bwd", C.byref(a), _s())


# ------------------------------------------------------------ conv module
def glu_dwconv_fwd(pre, w, out, B, T):
    C_ = w.shape[0]
    call("ste_glu_dwconv_fwd", ptr(pre), ptr(w), ptr(out), B, T, C_, w.shape[-1], _s())
    return out


def glu_dwconv_bwd(pre, w, dout, dpre, dw, B, T):
    C_ = w.shape[0]
    ws = _red_ws(pre.device, int(fn("ste_glu_dwconv_bwd_ws_floats")(B, T, C_, w.shape[-1]))) if dw is not None else None
    call("ste_glu_dwconv_bwd", ptr(pre), ptr(w), ptr(dout), ptr(dpre), ptr(dw), B, T, C_, w.shape[-1], *_ws_args(ws),
         _s())
    return dpre


# ------------------------------------------------------------------ fbank
def fbank(wav, lengths, Tmax, *, pad_value=1.0, mask_mode=0, feats=None, mask=None, work=None):
    """wav fp32 [B, N] (rows padded), lengths int32 [B] -> feats fp32 [B,Tmax,160], mask int64 [B,Tmax]."""
    B = wav.shape[0]
    dev = wav.device
    if feats is None:
        feats = torch.empty((B, Tmax, 160), device=dev, dtype=F32)
    if mask is None:
        mask = torch.empty((B, Tmax), device=dev, dtype=torch.int64)
    if work is None:
        work = torch.empty(B * 2 * Tmax * 80 + B * 160, device=dev, dtype=F32)
    # algorithmic bytes: the waveforms once, the stacked features and the mask
    nbytes = 4 * B * wav.shape[1] + _nb(feats) + _nb(mask)
    _traced("fbank", nbytes, lambda: call("ste_fbank", ptr(wav), wav.stride(0), ptr(lengths), B, Tmax,
                                          float(pad_value), ptr(feats), ptr(mask), int(mask_mode), ptr(work), _s()))
    return feats, mask


# ------------------------------------------------------------------ heads
def attn_pool_fwd(t, w2, b2, h, mask, B, L, weights, pooled, pooled_bf16=None):
    call("ste_attn_pool_fwd", ptr(t), ptr(w2), ptr(b2), ptr(h), ptr(mask), B, L, t.shape[-1], h.shape[-1],
         ptr(weights), ptr(pooled), ptr(pooled_bf16), _s())


def attn_pool_fwd_f32(t, w2, b2, h, mask, B, L, weights, pooled, pooled_bf16=None):
    """attn_pool_fwd on fp32 scorer activations t and fp32 states h (the text side)."""
    assert t.dtype == F32 and h.dtype == F32
    call("ste_attn_pool_fwd_f32", ptr(t), ptr(w2), ptr(b2), ptr(h), ptr(mask), B, L, t.shape[-1], h.shape[-1],
         ptr(weights), ptr(pooled), ptr(pooled_bf16), _s())


def attn_pool_bwd_f32(t, w2, h, weights, dpooled, B, L, dh, dz, dw2=None, db2=None, db1=None, mask=None):
    """attn_pool_bwd on fp32 t / h with an fp32 dz (no low half needed)."""
    assert t.dtype == F32 and h.dtype == F32 and dz.dtype == F32
    nwork = fn("ste_attn_pool_bwd_work_floats")(B, L, t.shape[-1])
    if nwork < 0:
        raise _lib.SteError(f"ste_attn_pool_bwd_work_floats failed with status {nwork}")
    work = torch.empty(nwork, device=t.device, dtype=F32)
    call("ste_attn_pool_bwd_f32", ptr(t), ptr(w2), ptr(h), ptr(weights), ptr(dpooled), ptr(mask), B, L, t.shape[-1],
         h.shape[-1], ptr(dh), ptr(dz), ptr(dw2), ptr(db2), ptr(db1), ptr(work), _s())


def attn_pool_bwd(t, w2, h, weights, dpooled, B, L, dh, dz, dw2=None, db2=None, db1=None, dz_lo=None, mask=None):
    """AttentivePooling backward: dh += ..., dz (bf16, + optional low half dz_lo), dw2/db2 and the
    first Linear's bias gradient db1 (fp32 column sums of dz) accumulated.  mask: the forward's
    int32 mask (masked positions get no score gradient, as masked_fill's backward)."""
    nwork = fn("ste_attn_pool_bwd_work_floats")(B, L, t.shape[-1])
    if nwork < 0:
        raise _lib.SteError(f"ste_attn_pool_bwd_work_floats failed with status {nwork}")
    work = torch.empty(nwork, device=t.device, dtype=F32)
    call("ste_attn_pool_bwd", ptr(t), ptr(w2), ptr(h), ptr(weights), ptr(dpooled), ptr(mask), B, L, t.shape[-1],
         h.shape[-1], ptr(dh), ptr(dz), ptr(dz_lo), ptr(dw2), ptr(db2), ptr(db1), ptr(work), _s())


def mean_pool_fwd(h, mask, B, L, cls, weights, pooled, pooled_bf16=None):
    if h.dtype == F32:
        call("ste_mean_pool_fwd_f32", ptr(h), ptr(mask), B, L, h.shape[-1], int(bool(cls)), ptr(weights), ptr(pooled),
             ptr(pooled_bf16), _s())
        return
    call("ste_mean_pool_fwd", ptr(h), ptr(mask), B, L, h.shape[-1], int(bool(cls)), ptr(weights), ptr(pooled),
         ptr(pooled_bf16), _s())


def weighted_pool_bwd(weights, dpooled, B, L, dh):
    call("ste_weighted_pool_bwd", ptr(weights), ptr(dpooled), B, L, dh.shape[-1], ptr(dh), _s())


def xattn1_fwd(q, k, v, mask, B, S, nh, probs, out, drop_p=0.0, seed=0):
    P = q.shape[-1]
    call("ste_xattn1_fwd", ptr(q), ptr(k), ptr(v), _ld(k), ptr(mask), B, S, P, nh, float((P // nh) ** -0.5),
         float(drop_p), int(seed) & (2**64 - 1), ptr(probs), ptr(out), _s())


def xattn1_bwd(q, k, v, probs, dout, B, S, nh, dq, dk, dv, drop_p=0.0, seed=0, colsum=None, mask=None):
    """dk/dv fp32: accumulated (+=).  dk/dv bf16: written, and the fp32 column sums of [dk | dv]
    are added into colsum [2P] (the fused key/value bias gradient) when given.  mask: the
    forward's int32 key mask (masked keys get no score gradient)."""
    if dk.dtype == BF16:
        return xattn_bwd(q, k, v, probs, dout, B, S, nh, dq, dk, dv, (seed,), drop_p=drop_p, colsum=colsum,
                         mask=mask)
    P = q.shape[-1]
    assert _ld(dk) == _ld(dv)
    call("ste_xattn1_bwd", ptr(q), ptr(k), ptr(v), _ld(k), ptr(probs), ptr(dout), ptr(mask), B, S, P, nh,
         float((P // nh) ** -0.5), float(drop_p), int(seed) & (2**64 - 1), ptr(dq), ptr(dk), ptr(dv), _ld(dk), _s())


def xattn_fwd(q, k, v, mask, B, S, nh, probs, out, seeds, drop_p=0.0):
    """len(seeds) query sets sharing K/V: q / out rows qi*B + b, probs [(qi*B + b)*nh + h]*S."""
    P = q.shape[-1]
    nq = len(seeds)
    assert q.shape[0] == nq * B and out.shape[0] == nq * B and probs.numel() >= nq * B * nh * S
    call("ste_xattn_fwd", ptr(q), ptr(k), ptr(v), _ld(k), ptr(mask), B, S, P, nh, nq, float((P // nh) ** -0.5),
         float(drop_p), int(seeds[0]) & (2**64 - 1), int(seeds[-1]) & (2**64 - 1), ptr(probs), ptr(out), _s())


def xattn_bwd(q, k, v, probs, dout, B, S, nh, dq, dk, dv, seeds, drop_p=0.0, colsum=None, mask=None):
    """dk/dv fp32: accumulated (+=).  dk/dv bf16: written (ste_xattn_bwd_bf16), and the fp32
    column sums of [dk | dv] are added into colsum [2P] when given."""
    P = q.shape[-1]
    nq = len(seeds)
    assert _ld(dk) == _ld(dv) and q.shape[0] == nq * B and dq.shape[0] == nq * B and dout.shape[0] == nq * B
    if dk.dtype == BF16:
        assert dv.dtype == BF16
        part = torch.empty(B, 2 * P, device=q.device, dtype=F32)
        call("ste_xattn_bwd_bf16", ptr(q), ptr(k), ptr(v), _ld(k), ptr(probs), ptr(dout), ptr(mask), B, S, P, nh, nq,
             float((P // nh) ** -0.5), float(drop_p), int(seeds[0]) & (2**64 - 1), int(seeds[-1]) & (2**64 - 1),
             ptr(dq), ptr(dk), ptr(dv), _ld(dk), ptr(part), _s())
        if colsum is not None:
            w = _red_ws(q.device, int(fn("ste_colsum_ws_floats")(B, 2 * P)))
            call("ste_colsum", ptr(part), 0, B, 2 * P, 2 * P, ptr(colsum), *_ws_args(w), _s())
        return
    assert colsum is None
    call("ste_xattn_bwd", ptr(q), ptr(k), ptr(v), _ld(k), ptr(probs), ptr(dout), ptr(mask), B, S, P, nh, nq,
         float((P // nh) ** -0.5), float(drop_p), int(seeds[0]) & (2**64 - 1), int(seeds[-1]) & (2**64 - 1),
         ptr(dq), ptr(dk), ptr(dv), _ld(dk), _s())


def align_attn_fwd(q, kv, kmask, B, L, T, nh, probs, out, drop_p=0.0, seed=0):
    P = kv.shape[-1] // 2
    call("ste_align_attn_fwd", ptr(q), _ld(q), ptr(kv), _ld(kv), ptr(kmask), B, L, T, P, nh, float(drop_p),
         int(seed) & (2**64 - 1), ptr(probs), ptr(out), _ld(out), _s())


def align_attn_bwd(q, kv, probs, dout, B, L, T, nh, dsbuf, dq, dkv, drop_p=0.0, seed=0):
    P = kv.shape[-1] // 2
    call("ste_align_attn_bwd", ptr(q), _ld(q), ptr(kv), _ld(kv), ptr(probs), ptr(dout), _ld(dout), B, L, T, P, nh,
         float(drop_p), int(seed) & (2**64 - 1), ptr(dsbuf), ptr(dq), _ld(dq), ptr(dkv), _ld(dkv), _s())


def rank1_bwd(a, w, z, act, out, dw=None, db=None):
    M, K = z.shape
    call("ste_rank1_bwd", ptr(a), ptr(w), ptr(z), M, K, int(act), ptr(out), ptr(dw), ptr(db), _s())


def l2norm_fwd(x, y, norms):
    call("ste_l2norm_fwd", ptr(x), x.shape[0], x.shape[1], ptr(y), ptr(norms), _s())


def l2norm_bwd(y, norms, dy, dx):
    call("ste_l2norm_bwd", ptr(y), ptr(norms), ptr(dy), y.shape[0], y.shape[1], ptr(dx), _s())


def similarity(a, t, S):
    call("ste_similarity", ptr(a), ptr(t), a.shape[0], t.shape[0], a.shape[1], ptr(S), _s())


def pair_loss_fwd(S, off_neg, align, B, L, tau, aw, gamma, s_pos, s_neg, loss):
    call("ste_pair_loss_fwd", ptr(S), _ld(S), off_neg, ptr(align), B, L, float(tau), float(aw), float(gamma),
         ptr(s_pos), ptr(s_neg), ptr(loss), _s())


def pair_loss_bwd(s_pos, s_neg, align, B, L, tau, aw, gamma, gscale, ds_pos, ds_neg, dalign=None):
    call("ste_pair_loss_bwd", ptr(s_pos), ptr(s_neg), ptr(align), B, L, float(tau), float(aw), float(gamma),
         ptr(gscale), ptr(ds_pos), ptr(ds_neg), ptr(dalign), _s())


def pair_sim_bwd(a, tp, tn, ds_pos, ds_neg, da, dtp, dtn):
    call("ste_pair_sim_bwd", ptr(a), ptr(tp), ptr(tn), ptr(ds_pos), ptr(ds_neg), a.shape[0], a.shape[1], ptr(da),
         ptr(dtp), ptr(dtn), _s())


def pair_metrics(S, off_neg, tau, acc, losses=None, loss_w=1.0):
    """acc fp64[6] += [Σ sigmoid(s_pos/τ), Σ sigmoid(s_neg/τ), Σ s_pos>s_neg, Σ top-1 hit, rows,
    loss_w·Σ losses] over S's rows (ste_pair_metrics)."""
    call("ste_pair_metrics", ptr(S), _ld(S), S.shape[0], int(off_neg), float(tau), ptr(losses),
         0 if losses is None else losses.numel(), float(loss_w), ptr(acc), _s())


def inbatch_ce(S, B, NB, row0, tau, weight, gscale, loss, dS):
    """In-batch-negative InfoNCE over the NB global clean transcripts: loss += ..., dS [B, NB] written."""
    call("ste_inbatch_ce", ptr(S), _ld(S), B, NB, int(row0), float(tau), float(weight), ptr(gscale), ptr(loss),
         ptr(dS), _ld(dS), _s())


def rowmat(X, Y, out, transpose_x=False):
    """out[R, P] += X·Y (or Xᵀ·Y) for small fp32 matrices (X [R, C] or [C, R], Y [C, P])."""
    if transpose_x:
        C, R = X.shape
        sxr, sxc = X.stride(1), X.stride(0)
    else:
        R, C = X.shape
        sxr, sxc = X.stride(0), X.stride(1)
    assert Y.shape[0] == C and Y.is_contiguous() and out.shape == (R, Y.shape[1]) and out.is_contiguous()
    call("ste_rowmat_f32", ptr(X), sxr, sxc, ptr(Y), R, C, Y.shape[1], ptr(out), _s())
    return out


# -------------------------------------------------------------- embedding
def text_embed_fwd(ids, pad_idx, word, pos, type0, out, pos_ids):
    B, L = ids.shape
    call("ste_text_embed_fwd", ptr(ids), B, L, word.shape[1], pad_idx, ptr(word), ptr(pos), ptr(type0), ptr(out),
         ptr(pos_ids), _s())


def text_embed_bwd(ids, pos_ids, dout, pad_idx, dword, dpos, dtype0):
    B, L = ids.shape
    ws = _red_ws(dout.device, int(fn("ste_text_embed_bwd_ws_floats")(B, L, dout.shape[-1]))) if dtype0 is not None \
        else None
    call("ste_text_embed_bwd", ptr(ids), ptr(pos_ids), ptr(dout), B, L, dout.shape[-1], pad_idx, ptr(dword),
         ptr(dpos), ptr(dtype0), *_ws_args(ws), _s())


# -------------------------------------------------------------- optimizer
SUMSQ_PARTS = 2048   # ste_sumsq's per-block fp64 partials (its grid is capped at 2048 blocks)


def sumsq(g, acc, part=None):
    """acc[0] += Σ g² (fp64); part (fp64 [SUMSQ_PARTS]): block sums added in block order."""
    if ATOMIC_SUMS:
        part = None
    assert part is None or (part.dtype == torch.float64 and part.numel() >= SUMSQ_PARTS)
    # algorithmic bytes: one fp32 read per gradient element (SURVEY §8d clip_grad_norm_)
    _traced("sumsq", 4 * g.numel(), lambda: call("ste_sumsq", ptr(g), g.numel(), ptr(acc), ptr(part), _s()))


def adamw(p, g, m, v, p_bf16, *, lr, beta1, beta2, eps, wd, step, sumsq_acc=None, max_norm=1.0):
    # algorithmic bytes (28 B/param): read p, g, m, v and write p, m, v in fp32, plus the
    # bf16 MFMA shadow of p when one is refreshed (2 B)
    nbytes = p.numel() * (28 + (2 if p_bf16 is not None else 0))
    _traced("adamw", nbytes, lambda: call("ste_adamw", ptr(p), ptr(g), ptr(m), ptr(v), ptr(p_bf16), p.numel(), float(lr),
                                          float(beta1), float(beta2), float(eps), float(wd), int(step), ptr(sumsq_acc),
                                          float(max_norm), _s()))


def cast_bf16(x, y):
    call("ste_cast_f32_bf16", ptr(x), ptr(y), x.numel(), _s())
    return y


def axpby(y, x, alpha=1.0, beta=1.0):
    """y = alpha*x + beta*y for fp32 2-D (or 1-D) views."""
    y2 = y if y.dim() == 2 else y.view(1, -1)
    x2 = x if x.dim() == 2 else x.view(1, -1)
    assert y2.shape == x2.shape and y.dtype == F32 and x.dtype == F32
    call("ste_axpby2d", ptr(y2), _ld(y2), ptr(x2), _ld(x2), y2.shape[0], y2.shape[1], float(alpha), float(beta), _s())
    return y


def copy2d(dst, src):
    assert dst.shape == src.shape and dst.dtype == src.dtype
    d2 = dst if dst.dim() == 2 else dst.view(1, -1)
    s2 = src if src.dim() == 2 else src.view(1, -1)
    call("ste_copy2d", ptr(d2), _ld(d2), ptr(s2), _ld(s2), d2.shape[0], d2.shape[1], dst.element_size(), _s())
    return dst


def spec_mask_fwd(x, spec, valid, embed):
    """x[r] = embed where spec[r] and valid[r] (x fp32 [rows, cols]; spec int32 [rows])."""
    call("ste_spec_mask_fwd", ptr(x), _ld(x), ptr(spec), ptr(valid), ptr(embed), x.shape[0], x.shape[1], _s())


def spec_mask_bwd(dx, spec, valid, dembed=None):
    """dembed += Σ dx[r] over the SpecAugment rows, and dx[r] = 0 there."""
    ws = _red_ws(dx.device, int(fn("ste_spec_mask_bwd_ws_floats")(dx.shape[0], dx.shape[1]))) if dembed is not None \
        else None
    call("ste_spec_mask_bwd", ptr(dx), _ld(dx), ptr(spec), ptr(valid), ptr(dembed), dx.shape[0], dx.shape[1],
         *_ws_args(ws), _s())


def transpose16(src, dst=None):
    """dst [cols, rows] = srcᵀ for a 2-D bf16 (2-byte) matrix with unit column stride."""
    assert src.dim() == 2 and src.stride(1) == 1 and src.element_size() == 2
    rows, cols = src.shape
    if dst is None:
        dst = torch.empty(cols, rows, device=src.device, dtype=src.dtype)
    assert dst.shape == (cols, rows) and dst.stride(1) == 1 and dst.dtype == src.dtype
    call("ste_transpose16", ptr(dst), _ld(dst), ptr(src), _ld(src), rows, cols, _s())
    return dst


def colsum(x, out):
    """out[c] += Σ_r x[r, c] (ordered partial sums: run-to-run deterministic)."""
    ws = _red_ws(x.device, int(fn("ste_colsum_ws_floats")(x.shape[0], x.shape[1])))
    call("ste_colsum", ptr(x), int(x.dtype == BF16), x.shape[0], x.shape[1], _ld(x), ptr(out), *_ws_args(ws), _s())
    return out


# ------------------------------------------------- row-sparse gradient exchange
def rows_extract(ids, pad_idx, grad2d, flags, out_ids, rows, count):
    """Unique non-pad ids -> out_ids (-1 padded), rows = grad2d[ids], grad2d[ids] = 0."""
    assert ids.dtype == torch.int64 and grad2d.dtype == F32 and rows.shape[0] == out_ids.numel()
    call("ste_rows_extract", ptr(ids), ids.numel(), int(pad_idx), ptr(grad2d), grad2d.shape[1], ptr(flags),
         ptr(out_ids), ptr(rows), out_ids.numel(), ptr(count), _s())


def rows_accumulate(grad2d, ids, rows, scale):
    """grad2d[ids[s]] += scale * rows[s] for ids[s] >= 0 (ids unique)."""
    call("ste_rows_accumulate", ptr(grad2d), grad2d.shape[1], ptr(ids), ptr(rows), ids.numel(), float(scale), _s())

