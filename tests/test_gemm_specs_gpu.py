"""Every compile-time epilogue of the persistent 8-phase bf16 GEMM (gemm.hip STE_EPI_SPECS), at the
shapes where the library plans that kernel — >= 240 tiles of 256x256 — against fp64 on the same
bf16 operands.

The end-to-end parity tests run B <= 4 (<= 96 tiles per encoder GEMM), where every encoder GEMM takes
the 128x128 gemm_bf16_kernel; the b = 64 bench runs these instantiations instead (c2 rows
M = 31,936).  The MX-fp8 kernel's scale-select bug hid for two rounds exactly there
(test_kernels_gpu.py::test_gemm_mx8_8ph_specs), so each case here:
  * asserts the kernel the library launched (ste_gemm_kernel_name, recorded by ops.GEMM_TRACE at the
    launch itself) is the intended gemm_8ph_kernel<A_KC, B_KC, EF, ACT> instantiation;
  * compares every output it writes (C, the pre-activation copy C2, the bf16 / low-half copy C3,
    the bias-gradient column sums) with the fp64 restatement of the epilogue (include/ste.h order:
    (acc + bias)·alpha -> C2 -> act -> ·act'(Z) -> ·dropout -> ·row_scale -> Σcol -> +R -> +beta·C);
  * dropout masks are rebuilt from the kernels' counter hash (kref.ste_hash, restated in torch
    int64 on the GPU and checked against the numpy form).
Shapes: the c2 layer shapes (M = 31,936 rows; N / K of the Conformer FFN, QKV, O / FFN-out, the
pointwise convs, the dX products) or the text encoder's (M = 8,192) for the XLM-R epilogues.
Bounds: fp32 outputs 1e-5 relative (fp32 accumulation order over K <= 4,096), bf16 outputs 4e-3
(one bf16 rounding, 2^-9 relative), hi + lo split copies 2e-5.  Each case prints its errors; the
collected lines are profiles/r6_parity.txt."""
import math

import numpy as np
import pytest
import torch

from kref import ste_hash

pytestmark = pytest.mark.gpu
DEV = "cuda"
C2M = 31936   # c2 audio rows: b = 64 clips x 499 frames
TXT = 8192    # c2 text rows: 2b x 64 tokens

SWISH, GELU, SWISH_BWD, GELU_BWD = 1, 2, 11, 12
EF_BIAS, EF_C2, EF_Z, EF_DROP, EF_RS, EF_COLSUM, EF_R = 1, 2, 4, 8, 16, 32, 64
EF_BETA, EF_CBF16, EF_C3 = 256, 512, 1024

# id: (A k-contiguous, B k-contiguous, EF, ACT, M, N, K, extra)  — the STE_EPI_SPECS list, in its order
# (extra: "lo" = the C3 copy is the low half v - bf16(v); "beta" / "rs" / "alpha" = run-time features
# that route to the generic EF = -1 instantiation)
SPECS = {
    "ffn_in_swish":        (True, True, EF_BIAS | EF_C2 | EF_CBF16, SWISH, C2M, 4096, 1024, ""),
    "xlmr_in_gelu":        (True, True, EF_BIAS | EF_C2 | EF_CBF16, GELU, TXT, 3072, 768, ""),
    "ffn_in_eval":         (True, True, EF_BIAS | EF_CBF16, SWISH, C2M, 4096, 1024, ""),
    "w2v_conv":            (True, True, EF_C2 | EF_CBF16, GELU, C2M, 512, 1536, ""),
    "w2v_conv_last":       (True, True, EF_C2, GELU, C2M, 512, 1024, ""),
    "postln_out_drop":     (True, True, EF_BIAS | EF_R | EF_DROP, 0, C2M, 768, 3072, ""),
    "w2v_ffn_in_drop":     (True, True, EF_BIAS | EF_C2 | EF_DROP | EF_CBF16, GELU, C2M, 3072, 768, ""),
    "gelu_bias_bf16":      (True, True, EF_BIAS | EF_CBF16, GELU, TXT, 3072, 768, ""),
    "text_qkv_precise":    (True, True, EF_BIAS | EF_C3, 0, TXT, 2304, 1536, ""),
    "text_ffn_in_precise": (True, True, EF_BIAS | EF_C2 | EF_C3 | EF_CBF16, GELU, TXT, 3072, 1536, "lo"),
    "ffn_out_residual":    (True, True, EF_BIAS | EF_R, 0, C2M, 1024, 4096, ""),
    "o_proj_residual":     (True, True, EF_BIAS | EF_R, 0, C2M, 1024, 1024, "alpha"),
    "qkv":                 (True, True, EF_BIAS | EF_CBF16, 0, C2M, 3072, 1024, ""),
    "pw_conv1":            (True, True, EF_CBF16, 0, C2M, 2048, 1024, ""),
    "pw_conv2_drop":       (True, True, EF_R | EF_DROP, 0, C2M, 1024, 1024, ""),
    "residual_only":       (True, True, EF_R, 0, C2M, 1024, 1024, ""),
    "dx_bf16":             (True, False, EF_CBF16, 0, C2M, 1024, 4096, ""),
    "dx_f32":              (True, False, 0, 0, C2M, 1024, 3072, ""),
    "dz_swish_colsum":     (True, True, EF_Z | EF_COLSUM | EF_CBF16, SWISH_BWD, C2M, 4096, 1024, ""),
    "dz_gelu_colsum":      (True, True, EF_Z | EF_COLSUM | EF_CBF16, GELU_BWD, TXT, 3072, 768, ""),
    "dz_gelu_colsum_c3":   (True, True, EF_Z | EF_COLSUM | EF_C3 | EF_CBF16, GELU_BWD, TXT, 3072, 1536, "lo"),
    "dz_gelu_c3":          (True, True, EF_Z | EF_C3 | EF_CBF16, GELU_BWD, TXT, 3072, 1536, "lo"),
    "dz_swish_frozen":     (True, True, EF_Z | EF_CBF16, SWISH_BWD, C2M, 4096, 1024, ""),
    "dz_gelu_frozen":      (True, True, EF_Z | EF_CBF16, GELU_BWD, TXT, 3072, 768, ""),
    "dz_gelu_colsum_drop": (True, True, EF_Z | EF_COLSUM | EF_DROP | EF_CBF16, GELU_BWD, C2M, 3072, 768, ""),
    "dz_gelu_drop":        (True, True, EF_Z | EF_DROP | EF_CBF16, GELU_BWD, C2M, 3072, 768, ""),
    "plain_f32":           (True, True, 0, 0, C2M, 1024, 1024, ""),
    # run-time features outside the list: the generic instantiation (EF = -1) of both layouts
    "generic_rs_beta":     (True, True, EF_BIAS | EF_RS | EF_BETA, 0, C2M, 1024, 1024, "beta"),
    "generic_dx_beta":     (True, False, EF_BETA, 0, C2M, 1024, 512, "beta"),
}
COMPILED = {k for k, v in SPECS.items() if v[7] != "beta"}

_M1, _M2, _M3 = 0x9E3779B97F4A7C15, 0xFF51AFD7ED558CCD, 0xC4CEB9FE1A85EC53


def _i64(u):
    return u - (1 << 64) if u >= 1 << 63 else u


def hash_t(seed, idx):
    """kref.ste_hash (murmur fmix64 of seed ^ idx·golden, low 32 bits) on int64 GPU tensors:
    two's-complement multiplies wrap like uint64, and the logical >> 33 is the arithmetic one masked."""
    x = idx * _i64(_M1)
    x = x ^ _i64(seed & ((1 << 64) - 1))
    x = x ^ ((x >> 33) & ((1 << 31) - 1))
    x = x * _i64(_M2)
    x = x ^ ((x >> 33) & ((1 << 31) - 1))
    x = x * _i64(_M3)
    x = x ^ ((x >> 33) & ((1 << 31) - 1))
    return x & 0xFFFFFFFF


def drop_scale_t(seed, p, M, N, ld):
    idx = torch.arange(M, device=DEV, dtype=torch.int64)[:, None] * ld + torch.arange(N, device=DEV)[None, :]
    # the kernels' threshold: (uint32)(float p · 2^32), from the fp32 drop_p of the argument block
    keep = hash_t(seed, idx) >= min(int(float(np.float32(p)) * 4294967296.0), 0xFFFFFFFF)
    return keep.double() / (1.0 - p)


def test_hash_restatement():
    """The torch restatement of the dropout hash equals kref's numpy one (itself the kernels')."""
    idx = np.concatenate([np.arange(4096), np.array([2**31 - 1, 2**32 + 5, 31936 * 4096 - 1])]).astype(np.uint64)
    for seed in (0, 99, 2**63 + 12345):
        want = ste_hash(seed, idx).astype(np.int64)
        got = hash_t(seed, torch.from_numpy(idx.astype(np.int64)).to(DEV)).cpu().numpy()
        assert np.array_equal(got, want), seed


def _act64(z, act):
    if act == SWISH:
        return z * torch.sigmoid(z)
    if act == GELU:
        return 0.5 * z * (1.0 + torch.erf(z / math.sqrt(2.0)))
    return z


def _actd64(z, act):
    if act == SWISH_BWD:
        sg = torch.sigmoid(z)
        return sg * (1.0 + z * (1.0 - sg))
    if act == GELU_BWD:
        return 0.5 * (1.0 + torch.erf(z / math.sqrt(2.0))) + z * torch.exp(-0.5 * z * z) / math.sqrt(2.0 * math.pi)
    return torch.ones_like(z)


def _rel(a, ref):
    a, ref = a.double(), ref.double()
    return ((a - ref).norm() / (ref.norm() + 1e-30)).item()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", list(SPECS))
def test_gemm_8ph_epilogue_spec(case):
    from speech_transcript_embeddings_amd import ops
    a_kc, b_kc, ef, act, M, N, K, extra = SPECS[case]
    g = torch.Generator(device=DEV).manual_seed(len(case) * 7919 + N)
    x = (torch.randn(M, K, device=DEV, generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) * (1.0 / math.sqrt(K))).bfloat16()
    kw = {}
    if ef & EF_BIAS:
        kw["bias"] = torch.randn(N, device=DEV, generator=g) * 0.1
    if ef & EF_C2:
        kw["pre_out"] = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    if ef & EF_C3:
        kw["out_bf16_copy"] = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        kw["copy_lo"] = extra == "lo"
    if ef & EF_Z:
        kw["z"] = (torch.randn(M, N, device=DEV, generator=g) * 1.5).bfloat16()
    if ef & EF_R:
        kw["residual"] = torch.randn(M, N, device=DEV, generator=g)
    if ef & EF_DROP:
        kw["drop_p"], kw["seed"] = 0.1, 0x5EED0000 + N
    if ef & EF_RS:
        kw["row_scale"] = (torch.rand(M, device=DEV, generator=g) > 0.25).float() * 0.75
    if ef & EF_COLSUM:
        kw["colsum"] = torch.zeros(N, device=DEV)
    c0 = None
    if ef & EF_BETA:
        c0 = torch.randn(M, N, device=DEV, generator=g)
        kw["out"], kw["beta"] = c0.clone(), 0.5
    alpha = 0.5 if extra == "alpha" else 1.0
    if act:
        kw["act"] = act
    out_bf16 = bool(ef & EF_CBF16)
    # dX layout: A = dY [M, K] k-contiguous, B = W k-major ([K, N]: the nn.Linear weight [out=K, in=N])
    bmat = w if b_kc else w.t().contiguous()
    ops.GEMM_TRACE = []
    try:
        y = ops.gemm(x, bmat, a_kc=True, b_kc=b_kc, M=M, N=N, K=K, out_bf16=out_bf16, alpha=alpha, **kw)
        torch.cuda.synchronize()
        names = [t[0] for t in ops.GEMM_TRACE]
    finally:
        ops.GEMM_TRACE = None
    want = "gemm_8ph_kernel<%s, %s, %d, %d>" % (str(a_kc).lower(), str(b_kc).lower(),
                                                 ef if case in COMPILED else -1, act if case in COMPILED else 0)
    assert names == [want], (names, want)

    v = x.double() @ w.double().t()
    if "bias" in kw:
        v = v + kw["bias"].double()
    v = v * alpha
    z_pre = v
    if act in (SWISH, GELU):
        v = _act64(v, act)
    if act in (SWISH_BWD, GELU_BWD):
        v = v * _actd64(kw["z"].double(), act)
    if ef & EF_DROP:
        v = v * drop_scale_t(kw["seed"], kw["drop_p"], M, N, N)
    if ef & EF_RS:
        v = v * kw["row_scale"].double()[:, None]
    csum = v.sum(0) if ef & EF_COLSUM else None
    if ef & EF_R:
        v = v + kw["residual"].double()
    if c0 is not None:
        v = v + 0.5 * c0.double()
    errs = {}
    errs["C"] = _rel(y, v)
    bound_c = 4e-3 if out_bf16 else 1e-5
    if ef & EF_C2:
        errs["C2"] = _rel(kw["pre_out"], z_pre)
    if ef & EF_C3:
        if kw["copy_lo"]:   # C + C3 = hi + lo of the fp32 value (~16 mantissa bits)
            errs["C+C3"] = _rel(y.double() + kw["out_bf16_copy"].double(), v)
        else:
            errs["C3"] = _rel(kw["out_bf16_copy"], v)
    if csum is not None:
        errs["colsum"] = _rel(kw["colsum"], csum)
    print(f"[r6 gemm spec] {case:22s} {want:40s} M={M} N={N} K={K} tiles={((M + 255) // 256) * ((N + 255) // 256)} "
          + " ".join(f"{k}={e:.2e}" for k, e in errs.items()))
    assert errs["C"] < bound_c, errs
    if "C2" in errs:
        assert errs["C2"] < 4e-3, errs
    if "C3" in errs:
        assert errs["C3"] < 4e-3, errs
    if "C+C3" in errs:
        assert errs["C+C3"] < 2e-5, errs
    if "colsum" in errs:
        assert errs["colsum"] < 1e-4, errs


@pytest.mark.timeout(300)
@pytest.mark.parametrize("M,N,K", [(4096, 1024, C2M), (1024, 4096, C2M), (3072, 1024, C2M), (1024, 1024, C2M),
                                   (768, 3072, TXT)])
def test_gemm_8ph_weight_gradient_c2(M, N, K):
    """The c2 weight gradients dW += dYᵀ·X (both operands k-major, K = the 31,936 audio rows or the
    8,192 text rows) on gemm_8ph_kernel<false, false, 0, 0> split-K slabs + the ordered slab
    reduction, as the step plans them (80 MB workspace), against fp64."""
    from speech_transcript_embeddings_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + N)
    dy = (torch.randn(K, M, device=DEV, generator=g) * 0.1).bfloat16()
    xx = torch.randn(K, N, device=DEV, generator=g).bfloat16()
    ws = torch.empty(80 << 18, device=DEV)
    acc = torch.randn(M, N, device=DEV, generator=g)
    out = acc.clone()
    ops.GEMM_TRACE = []
    try:
        ops.linear_dw(dy, xx, out=out, beta=1.0, ws=ws)
        torch.cuda.synchronize()
        names = [t[0] for t in ops.GEMM_TRACE]
    finally:
        ops.GEMM_TRACE = None
    assert names == ["gemm_8ph_kernel<false, false, 0, 0>"], names
    ref = dy.double().t() @ xx.double() + acc.double()
    e = _rel(out, ref)
    print(f"[r6 gemm spec] dW M={M} N={N} K={K} C={e:.2e}")
    assert e < 1e-5, e
