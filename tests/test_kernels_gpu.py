"""Per-kernel parity: every libste.so kernel vs a plain PyTorch fp32 reference of the same op
(tests/kref.py), through the C ABI (speech_transcript_embeddings_amd.ops -> ctypes)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from kref import attention_ref, drop_scale, glu_dwconv_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from speech_transcript_embeddings_amd import ops as _ops
    return _ops


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# ------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(64, 128, 64), (300, 384, 200), (1000, 1024, 160), (130, 776, 96),
                                   # >= 240 256x256 tiles: the global_load_lds kernel (fwd KC.KC / dX KC.KM)
                                   (4000, 4096, 512), (3999, 512, 4096), (3000, 5128, 256)])
def test_gemm_layouts(ops, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    b = torch.randn(N, device=DEV)
    y = ops.linear(x, w, b)
    assert rel_err(y, x.float() @ w.float().t() + b) < 1e-5
    dy = torch.randn(M, N, device=DEV).bfloat16()
    assert rel_err(ops.linear_dx(dy, w), dy.float() @ w.float()) < 1e-5
    assert rel_err(ops.linear_dw(dy, x), dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(1, 1, 8), (7, 3, 72), (100, 5, 1024), (333, 1, 768), (2, 24, 8)])
def test_gemm_tiny_shapes(ops, M, N, K):
    """The edges of the GEMM contract: one row, one to five output columns (N < 8: the element-wise
    epilogue tail; e.g. the attention-pooling scorer's single logit), the minimum K of 8; fp32 and
    bf16 outputs, with and without bias."""
    torch.manual_seed(M * 31 + N)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    b = torch.randn(N, device=DEV)
    ref = x.double() @ w.double().t()
    assert rel_err(ops.linear(x, w, b), ref + b.double()) < 1e-6
    assert rel_err(ops.linear(x, w, None, out_bf16=True), ref) < 4e-3


@pytest.mark.parametrize("rows,cols", [(1024, 4096), (3072, 1024), (130, 77), (64, 1), (1000, 4100)])
def test_transpose16(ops, rows, cols):
    x = torch.randn(rows, cols, device=DEV).bfloat16()
    assert torch.equal(ops.transpose16(x), x.t().contiguous())
    big = torch.randn(rows, cols + 8, device=DEV).bfloat16()[:, 3:3 + cols]  # strided source view
    assert torch.equal(ops.transpose16(big), big.t().contiguous())


def test_dx_through_cached_transpose():
    """dX = dY·W on the KC kernel with ParamStore.wt equals the k-major kernel bit for bit, and
    the cached Wᵀ follows optimizer steps (trained weights) but is reused for frozen ones."""
    import json
    from conftest import GOLDEN
    from test_model_gpu import mini_model
    from speech_transcript_embeddings_amd import ops
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    meta = json.loads((GOLDEN / "model_golden_noalign.json").read_text())
    model = mini_model(meta)
    st = model.store
    trained = "audio_encoder.encoder.layers.1.ffn1.intermediate_dense.weight"
    frozen = "audio_encoder.encoder.layers.0.ffn1.intermediate_dense.weight"
    assert st.slots[trained].segment == "enc" and st.slots[frozen].segment == "frozen"
    dy = torch.randn(300, st.slots[trained].shape[0], device=DEV).bfloat16()
    for n in (trained, frozen):
        a = ops.linear_dx(dy, st.w(n), out_bf16=True)
        b = ops.linear(dy, st.wt(n), out_bf16=True)
        assert torch.equal(a, b)
    q = "audio_encoder.encoder.layers.1.self_attn.linear_q.weight"
    assert torch.equal(st.wt(q, 3), st.fused(q, 3, "w").t())
    t_frozen, t_trained = st.wt(frozen), st.wt(trained).clone()
    step = TrainStep(model, lr=1e-2, warmup=1, total_steps=10)
    data = synthetic_batch(2, 16000, 12, vocab=meta["mini"]["text"]["vocab_size"], seed=1)
    step(*data)
    step(*data)
    assert st.wt(frozen) is t_frozen  # frozen: built once
    assert not torch.equal(st.wt(trained), t_trained)  # trained: follows the optimizer
    assert torch.equal(st.wt(trained), st.w(trained).t())
    with torch.no_grad():  # a write outside the optimizer (e.g. load_state_dict) invalidates it
        model.get_parameter(frozen).mul_(2.0)
    st.sync_shadow()
    assert torch.equal(st.wt(frozen), st.w(frozen).t())


@pytest.mark.parametrize("M,N,K,ws_mb", [(4096, 1024, 31936, 80),   # c2 FFN intermediate dW: S=4, 3 leftover K-tiles on slabs 0-2
                                         (1024, 1024, 31936, 80),   # c2 O-proj dW: S=16, Kc=31, 3 leftover K-tiles
                                         (1024, 1024, 15968, 80),   # c3 (b=32) O-proj dW: S=16, ragged 32-row tail
                                         (3072, 768, 8192, 80),     # text QKV dW over 2bL rows
                                         (768, 768, 31936, 80),     # 9 tiles: S=28 > 16, the reduce's loop tail
                                         (1032, 520, 4160, 8),      # ragged M/N tiles; workspace caps S at 3
                                         (2048, 1024, 960, 80)])    # K < 16 tiles: no split
def test_gemm_dw_splitk(ops, M, N, K, ws_mb):
    """Weight gradient dW += dYᵀ·X (both operands k-major) through the split-K 8-phase path."""
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(K)
    dy = torch.randn(K, M, device=DEV).bfloat16()
    x = torch.randn(K, N, device=DEV).bfloat16()
    ws = torch.empty(ws_mb << 18, device=DEV)
    g = torch.randn(M, N, device=DEV)
    ref = dy.float().t() @ x.float() * 0.5 + g
    out = g.clone()
    ops.linear_dw(dy, x, out=out, beta=1.0, alpha=0.5, ws=ws)
    assert rel_err(out, ref) < 1e-5
    args = _lib.GemmArgs(M=M, N=N, K=K, batch=1, a_kc=0, b_kc=0, A=1, B=1, C=1, ldc=N, lda=M, ldb=N, alpha=1.0,
                         ws=1, ws_bytes=ws.numel() * 4)
    kern = int(_lib.fn("ste_gemm_kernel")(__import__("ctypes").byref(args)))
    assert (kern >= 12) == (K >= 16 * 64), kern


@pytest.mark.parametrize("M,K", [(8192, 6144),   # text FFN-out, split-bf16 forward: 96 tiles, 2 x 48 K-tiles
                                 (8192, 3072),   # text FFN-in input gradient into the residual gradient
                                 (4000, 2624)])  # ragged M; 41 K-tiles: slab 0 takes the leftover one
def test_gemm_few_tile_splitk(ops, M, K):
    """Outputs too narrow for the CUs (N = 768, <= 128 tiles of 256x256) with a workspace run as 2
    K-slabs on the 8-phase kernel + a reduction that applies the generic epilogue: same results
    as the fp32 reference and the dropout mask of the tile epilogue (same hash of row, col)."""
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(K)
    N = 768
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV)
    ws = torch.empty(80 << 18, device=DEV)
    mm = x.float() @ w.float().t()
    seed, p = 99, 0.1
    idx = (np.arange(M)[:, None] * N + np.arange(N)[None, :]).astype(np.uint64)
    dmask = torch.from_numpy(drop_scale(seed, idx, p)).to(DEV)
    # bias + residual + dropout, fp32 out (the post-LN FFN-out / O-proj)
    y = ops.linear(x, w, b, residual=r, drop_p=p, seed=seed, ws=ws)
    assert rel_err(y, (mm + b) * dmask + r) < 1e-5
    y0 = ops.linear(x, w, b, residual=r, drop_p=p, seed=seed)          # no workspace: one-slab kernel
    assert torch.equal((y - r) == 0, (y0 - r) == 0)                     # identical dropout mask
    assert rel_err(y, y0) < 1e-6
    # GELU with the bf16 pre-activation, bf16 out; activation backward with Z; beta accumulate
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    h = ops.linear(x, w, b, act=_lib.ACT_GELU, pre_out=pre, out_bf16=True, ws=ws)
    assert rel_err(h, F.gelu(mm + b)) < 5e-3 and rel_err(pre, mm + b) < 5e-3
    z = torch.randn(M, N, device=DEV).bfloat16()
    c = torch.randn(M, N, device=DEV)
    c0 = c.clone()
    ops.linear(x, w, None, act=_lib.ACT_GELU_BWD, z=z, beta=1.0, out=c, alpha=0.5, ws=ws)
    zf = z.float()
    gd = torch.special.ndtr(zf) + zf * torch.exp(-0.5 * zf * zf) / math.sqrt(2 * math.pi)
    assert rel_err(c, 0.5 * mm * gd + c0) < 1e-5
    args = _lib.GemmArgs(M=M, N=N, K=K, batch=1, a_kc=1, b_kc=1, A=1, B=1, C=1, ldc=N, lda=K, ldb=K, alpha=1.0,
                         ws=1, ws_bytes=ws.numel() * 4)
    assert int(_lib.fn("ste_gemm_kernel")(__import__("ctypes").byref(args))) == 12   # split-K family


@pytest.mark.parametrize("B,To,k,st", [(24, 1100, 3, 2),    # 17 whole K-tiles + a 12-frame tail
                                       (32, 1024, 2, 2)])   # K a multiple of 64: no tail launch
def test_gemm_batched_dw_strided(ops, B, To, k, st):
    """wav2vec2 conv-stack weight gradient: per-clip dW slabs dz_bᵀ·X_b over the strided im2col
    view of each clip (both operands k-major, batch = clips) on the 8-phase kernel + the small
    kernel's ragged-K tail, against fp32 per clip."""
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(To)
    cin, cout = 512, 512
    Ti = (To - 1) * st + k
    dz = torch.randn(B * To, cout, device=DEV).bfloat16()
    hin = torch.randn(B * Ti, cin, device=DEV).bfloat16()
    b = torch.as_strided(hin, (To, k * cin), (st * cin, 1))
    part = torch.empty(B * cout, k * cin, device=DEV)
    ops.gemm(dz, b, a_kc=False, b_kc=False, M=cout, N=k * cin, K=To, batch=B, stride_a=To * cout,
             stride_b=Ti * cin, stride_c=cout * k * cin, out=part)
    for i in (0, B // 2, B - 1):
        xi = torch.as_strided(hin, (To, k * cin), (st * cin, 1), i * Ti * cin).float()
        ref = dz[i * To:(i + 1) * To].float().t() @ xi
        assert rel_err(part[i * cout:(i + 1) * cout], ref) < 1e-5, i
    args = _lib.GemmArgs(M=cout, N=k * cin, K=To, batch=B, a_kc=0, b_kc=0, A=1, B=1, C=1, ldc=k * cin, lda=cout,
                         ldb=st * cin, alpha=1.0)
    assert int(_lib.fn("ste_gemm_kernel")(__import__("ctypes").byref(args))) == 8 + 3   # 8-phase, KM x KM


def _mx8_dequant(q, sc):
    """e4m3 bytes + E8M0 block scales -> fp64 (torch's float8_e4m3fn is the OCP encoding)."""
    v = q.view(torch.float8_e4m3fn).double()
    e = sc.long().repeat_interleave(32, dim=1) - 127
    return v * torch.pow(2.0, e.double())


# the last three have >= 240 256x256 tiles: the persistent 8-phase MX kernel (ragged M, N = 4096)
@pytest.mark.parametrize("M,N,K", [(1000, 768, 1024), (4000, 3072, 1024), (2000, 1024, 4096), (300, 2048, 128),
                                   (8000, 2048, 1024), (6000, 3072, 2048), (4100, 4096, 1024)])
def test_gemm_mx8(ops, M, N, K):
    """MX-fp8 GEMM (config 5): exact on the dequantised operands (fp32 accumulation), quantiser
    bit-exact against torch's e4m3 cast with the same block scale, and a few % from bf16."""
    torch.manual_seed(8)
    x = (torch.randn(M, K, device=DEV) * torch.rand(M, 1, device=DEV) * 4).bfloat16()
    x[3, 64:96] = 0  # a zero block
    w = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    xq = ops.mx8_quant(x)
    wq = ops.mx8_quant(w)
    # quantiser: e = ceil(log2(amax/448)) per 32-block, q = e4m3(x / 2^e)
    xb = x.float().view(M, K // 32, 32)
    amax = xb.abs().amax(-1)
    e = torch.where(amax > 0, torch.ceil(torch.log2(amax / 448.0)), torch.full_like(amax, -127.0)).clamp(-127, 127)
    assert torch.equal(xq[1].long() - 127, e.long())
    qref = (xb / torch.pow(2.0, e).unsqueeze(-1)).view(M, K).to(torch.float8_e4m3fn).view(torch.uint8)
    assert (xq[0] != qref).float().mean().item() < 1e-4
    ref = _mx8_dequant(*xq) @ _mx8_dequant(*wq).T
    y = ops.linear_mx8(xq, wq)
    assert rel_err(y.double(), ref) < 1e-4  # fp32 accumulation order (1.5e-5 measured at K=1024)
    ybf = x.double() @ w.double().T
    assert rel_err(y.double(), ybf) < 5e-2
    # epilogue options ride on the fp32 accumulators unchanged: bias + swish + pre-activation
    bias = torch.randn(N, device=DEV)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    yb = ops.linear_mx8(xq, wq, bias, act=1, out_bf16=True, pre_out=pre)
    z = ref + bias.double()
    assert rel_err(pre.double(), z) < 1e-2
    assert rel_err(yb.double(), z * torch.sigmoid(z)) < 1e-2
    # fp8 output of the epilogue (the FFN intermediate feeding the next MX-fp8 GEMM) equals the
    # quantiser applied to the fp32 output; out=False writes only the fp8 copy
    yf = torch.empty(M, N, device=DEV)
    q = (torch.empty(M, N, device=DEV, dtype=torch.uint8), torch.empty(M, N // 32, device=DEV, dtype=torch.uint8))
    ops.linear_mx8(xq, wq, bias, act=1, out=yf, q_out=q)
    qr = ops.mx8_quant(yf.bfloat16())  # reference quantiser (bf16 input: compare dequantised values)
    assert rel_err(_mx8_dequant(*q), yf.double()) < 4e-2
    assert (q[1].long() - qr[1].long()).abs().max().item() <= 1
    q2 = (torch.zeros_like(q[0]), torch.zeros_like(q[1]))
    assert ops.linear_mx8(xq, wq, bias, act=1, out=False, q_out=q2) is q2
    assert torch.equal(q2[0], q[0]) and torch.equal(q2[1], q[1])


# every compile-time epilogue of the persistent 8-phase MX kernel (STE_MX8_SPECS) at >= 240 tiles,
# the shapes where the library takes that kernel: against the dequantised operands in fp64 (round
# 5: its scale-select bug had made 3/4 of every tile ~0 since round 3, unseen because no test
# reached these epilogues; libste_ab.so + STE_MX8_8PH=0 runs the same checks on the single-stage
# kernel)
@pytest.mark.parametrize("spec", ["bias_bf16", "bf16", "bias_r", "ffn_in_q8", "ffn_in_q8_noc", "dz"])
def test_gemm_mx8_8ph_specs(ops, spec):
    import ctypes
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(10)
    M, K = 16000, 1024
    N = 4096 if spec.startswith("ffn_in") else 1024
    x = (torch.randn(M, K, device=DEV) * 0.5).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    xq, wq = ops.mx8_quant(x), ops.mx8_quant(w)
    v = _mx8_dequant(*xq) @ _mx8_dequant(*wq).T
    bias = torch.randn(N, device=DEV)
    kw, q = {}, None
    if spec == "bias_bf16":
        kw = dict(bias=bias, out_bf16=True)
        ref = v + bias.double()
    elif spec == "bf16":
        kw = dict(out_bf16=True)
        ref = v
    elif spec == "bias_r":
        r = torch.randn(M, N, device=DEV)
        kw = dict(bias=bias, residual=r)
        ref = v + bias.double() + r.double()
    elif spec.startswith("ffn_in"):
        pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        q = (torch.empty(M, N, device=DEV, dtype=torch.uint8), torch.empty(M, N // 32, device=DEV, dtype=torch.uint8))
        kw = dict(bias=bias, act=_lib.ACT_SWISH, out_bf16=True, pre_out=pre, q_out=q)
        if spec.endswith("noc"):
            kw["out"] = False
        zz = v + bias.double()
        ref = zz * torch.sigmoid(zz)
    else:
        z = torch.randn(M, N, device=DEV).bfloat16()
        kw = dict(act=_lib.ACT_SWISH_BWD, z=z, out_bf16=True)
        zz = z.double()
        sg = torch.sigmoid(zz)
        ref = v * sg * (1 + zz * (1 - sg))
    args = _lib.GemmArgs(M=M, N=N, K=K, batch=1, a_kc=1, b_kc=1, A=1, B=1, lda=K, ldb=K, ldc=N, alpha=1.0,
                         C=0 if kw.get("out") is False else 1, c_bf16=int(bool(kw.get("out_bf16"))),
                         bias=1 if "bias" in kw else 0, R=1 if "residual" in kw else 0, ldr=N,
                         C2=1 if "pre_out" in kw else 0, ldc2=N, Z=1 if "z" in kw else 0, ldz=N,
                         act=kw.get("act", 0))
    eight = int(_lib.fn("ste_gemm_mx8_kernel")(ctypes.byref(args), int(q is not None)))
    assert eight == (0 if _lib.ab_env("STE_MX8_8PH", "1") == "0" else 1), eight
    y = ops.linear_mx8(xq, wq, **kw)
    if y is not False and kw.get("out") is not False:
        assert rel_err(y.double(), ref) < (1e-2 if kw.get("out_bf16") else 1e-4), spec
    if spec.startswith("ffn_in"):
        if not spec.endswith("noc"):
            assert rel_err(pre.double(), v + bias.double()) < 1e-2
        assert rel_err(_mx8_dequant(*q), ref) < 5e-2


# the opt-in MX-fp8 input gradient (engine.fp8_bwd): dz = (dY·W) ⊙ swish'(z) with z bf16, on the
# single-stage kernel (128 tiles) and the persistent 8-phase one (252 tiles); the dX operand pair
# is dY quantised along its row and Wᵀ (ParamStore.wtq) quantised along `out`
@pytest.mark.parametrize("M", [8000, 16000])
def test_gemm_mx8_act_bwd(ops, M):
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(9)
    N, K = 1024, 4096   # the dz GEMM's shape class: K = the FFN width, N = its output
    dh = (torch.randn(M, K, device=DEV) * 0.1).bfloat16()
    wt = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()   # Wᵀ as the MX B operand [N, K]
    z = torch.randn(M, N, device=DEV).bfloat16()
    dq, wq = ops.mx8_quant(dh), ops.mx8_quant(wt)
    out = ops.linear_mx8(dq, wq, act=_lib.ACT_SWISH_BWD, z=z, out_bf16=True)
    v = _mx8_dequant(*dq) @ _mx8_dequant(*wq).T
    zz = z.double()
    sg = torch.sigmoid(zz)
    ref = v * sg * (1 + zz * (1 - sg))
    assert rel_err(out.double(), ref) < 1e-2
    assert rel_err(out.double(), (dh.double() @ wt.double().T) * sg * (1 + zz * (1 - sg))) < 6e-2


def test_layernorm_mx8_output(ops):
    """LN forward's fused MX-fp8 copy (fp8_gemm: the LN feeding a Conformer Linear): scales are
    ceil(log2(amax/448)) of the fp32 output's 32-column blocks, payload = e4m3(y / 2^e)."""
    torch.manual_seed(6)
    rows, cols = 777, 1024
    x = torch.randn(rows, cols, device=DEV) * 3 + 1
    g, b = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV) * 0.1
    y = torch.empty(rows, cols, device=DEV)
    q = (torch.empty(rows, cols, device=DEV, dtype=torch.uint8),
         torch.empty(rows, cols // 32, device=DEV, dtype=torch.uint8))
    ops.layernorm_fwd(x, g, b, 1e-5, y=y, q8=q, act=1)
    yb = y.view(rows, cols // 32, 32)
    amax = yb.abs().amax(-1)
    e = torch.where(amax > 0, torch.ceil(torch.log2(amax / 448.0)), torch.full_like(amax, -127.0)).clamp(-127, 127)
    assert torch.equal(q[1].long() - 127, e.long())
    qref = (yb / torch.pow(2.0, e).unsqueeze(-1)).view(rows, cols).to(torch.float8_e4m3fn).view(torch.uint8)
    assert (q[0] != qref).float().mean().item() < 1e-4
    assert rel_err(_mx8_dequant(*q), y.double()) < 4e-2


def test_gemm_epilogues(ops):
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(1)
    M, N, K = 257, 256, 128
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16() * 0.1
    b = torch.randn(N, device=DEV)
    ref = x.float() @ w.float().t() + b
    for act, fn in [(_lib.ACT_SWISH, F.silu), (_lib.ACT_GELU, F.gelu), (_lib.ACT_TANH, torch.tanh),
                    (_lib.ACT_RELU, F.relu)]:
        pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        out = ops.linear(x, w, b, act=act, pre_out=pre)
        assert rel_err(out, fn(ref)) < 1e-5
        assert rel_err(pre, ref) < 5e-3
    # activation backward with Z, dropout, row scale, colsum, residual, beta
    z = torch.randn(M, N, device=DEV).bfloat16()
    rs = (torch.rand(M, device=DEV) > 0.3).float()
    r = torch.randn(M, N, device=DEV)
    cs = torch.zeros(N, device=DEV)
    c = torch.randn(M, N, device=DEV)
    c0 = c.clone()
    seed, p = 1234, 0.25
    ops.linear(x, w, None, act=_lib.ACT_GELU_BWD, z=z, drop_p=p, seed=seed, row_scale=rs, colsum=cs, residual=r,
               beta=1.0, out=c, alpha=0.5)
    idx = (np.arange(M)[:, None] * N + np.arange(N)[None, :]).astype(np.uint64)
    dmask = torch.from_numpy(drop_scale(seed, idx, p)).to(DEV)
    zf = z.float()
    gd = torch.special.ndtr(zf) + zf * torch.exp(-0.5 * zf * zf) / math.sqrt(2 * math.pi)
    v = 0.5 * (x.float() @ w.float().t()) * gd * dmask * rs[:, None]
    assert rel_err(cs, v.sum(0)) < 1e-4
    assert rel_err(c, v + r + c0) < 1e-5


# ------------------------------------------------ fp32 GEMM of the heads (ste_gemm_f32)
def _rel64(a, ref):
    a, ref = a.double(), ref.double()
    return ((a - ref).norm() / (ref.norm() + 1e-30)).item()


@pytest.mark.parametrize("M,N,K", [(64, 1536, 768), (128, 768, 1536), (8192, 384, 768), (37, 68, 52), (3, 8, 4)])
def test_gemm_f32_layouts(ops, M, N, K):
    """fp32 operands on the f32 matrix core (exact fmaf chains): forward, dX and dW layouts at
    the heads' shapes (projection / fusion at batch rows, the text pooling scorer at 2·b·L rows)
    and ragged ones, against float64."""
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV)
    b = torch.randn(N, device=DEV)
    assert _rel64(ops.linear(x, w, b), x.double() @ w.double().t() + b.double()) < 2e-6
    dy = torch.randn(M, N, device=DEV)
    assert _rel64(ops.linear_dx(dy, w), dy.double() @ w.double()) < 2e-6
    g = torch.randn(N, K, device=DEV)
    ref = g.double() + dy.double().t() @ x.double()
    ws = torch.empty(8 << 20, device=DEV)
    ops.linear_dw(dy, x, out=g, beta=1.0, ws=ws)    # K = M rows: split into slabs when M >= 1024
    assert _rel64(g, ref) < 2e-6
    # bit-for-bit repeatable (slabs summed in order, no atomics)
    g2 = torch.zeros(N, K, device=DEV)
    g3 = torch.zeros(N, K, device=DEV)
    ops.linear_dw(dy, x, out=g2, beta=1.0, ws=ws)
    ops.linear_dw(dy, x, out=g3, beta=1.0, ws=ws)
    assert torch.equal(g2, g3)


def test_gemm_f32_epilogues_and_views(ops):
    """Every epilogue option of the fp32 GEMM (bias, activation + fp32 pre-activation, activation
    backward with fp32 Z, dropout, row scale, column sums, residual, beta, bf16 copy) and strided
    operand / output views (the fusion input [proj | att] and its halves)."""
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(2)
    M, N, K = 130, 256, 192
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.1
    b = torch.randn(N, device=DEV)
    ref = x.double() @ w.double().t() + b.double()
    for act, fn in [(_lib.ACT_SWISH, F.silu), (_lib.ACT_GELU, F.gelu), (_lib.ACT_TANH, torch.tanh),
                    (_lib.ACT_RELU, F.relu)]:
        pre = torch.empty(M, N, device=DEV)
        c3 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        out = ops.linear(x, w, b, act=act, pre_out=pre, out_bf16_copy=c3)
        assert _rel64(out, fn(ref)) < 1e-5
        assert _rel64(pre, ref) < 2e-6
        assert torch.equal(c3, out.bfloat16())
    z = torch.randn(M, N, device=DEV)
    rs = (torch.rand(M, device=DEV) > 0.3).float()
    r = torch.randn(M, N, device=DEV)
    cs = torch.zeros(N, device=DEV)
    c = torch.randn(M, N, device=DEV)
    c0 = c.clone()
    seed, p = 99, 0.25
    ops.linear(x, w, None, act=_lib.ACT_GELU_BWD, z=z, drop_p=p, seed=seed, row_scale=rs, colsum=cs, residual=r,
               beta=1.0, out=c, alpha=0.5)
    idx = (np.arange(M)[:, None] * N + np.arange(N)[None, :]).astype(np.uint64)
    dmask = torch.from_numpy(drop_scale(seed, idx, p)).to(DEV).double()
    zf = z.double()
    gd = torch.special.ndtr(zf) + zf * torch.exp(-0.5 * zf * zf) / math.sqrt(2 * math.pi)
    v = 0.5 * (x.double() @ w.double().t()) * gd * dmask * rs.double()[:, None]
    assert _rel64(cs, v.sum(0)) < 1e-5
    assert _rel64(c, v + r.double() + c0.double()) < 1e-5
    # strided views: A = the right half of a [M, 2K] buffer, C = the right half of [M, 2N]
    big = torch.randn(M, 2 * K, device=DEV)
    cat = torch.zeros(M, 2 * N, device=DEV)
    ops.linear(big[:, K:], w, b, out=cat[:, N:])
    assert _rel64(cat[:, N:], big[:, K:].double() @ w.double().t() + b.double()) < 2e-6
    assert cat[:, :N].abs().max().item() == 0.0
    dyv = torch.randn(M, 2 * N, device=DEV)[:, N:]
    gw = torch.zeros(N, K, device=DEV)
    ops.linear_dw(dyv, x, out=gw, beta=1.0)
    assert _rel64(gw, dyv.double().t() @ x.double()) < 2e-6


# ------------------------- split-bf16 ("bf16x3") GEMM and fp32 attention: the precise text forward
def test_split_bf16_and_linear_x2(ops):
    """ste_split_bf16 writes [hi | lo] (and [hi | lo | hi]) images exactly, and one bf16 MFMA GEMM over
    the 2K concatenated columns of [x_hi | x_lo]·[w | w]ᵀ equals the product of the fp32 activations
    with the bf16-rounded weight to ~2^-16 (plain bf16 operands: ~2^-9), under every epilogue the
    text layer uses (bias + GELU + pre-activation + bf16 copy + dropout; residual)."""
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(11)
    M, N, K = 8192, 3072, 768
    x = torch.randn(M, K, device=DEV) + 2.0          # a common component, as LayerNorm outputs have
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    hi = x.bfloat16()
    lo = (x - hi.float()).bfloat16()
    a3 = ops.split_bf16(x, 3, 2)
    assert torch.equal(a3[:, :K], hi) and torch.equal(a3[:, K:2 * K], lo) and torch.equal(a3[:, 2 * K:], hi)
    a2 = ops.split_bf16(x, 2, 2)
    assert torch.equal(a2[:, :K], hi) and torch.equal(a2[:, K:], lo)
    w2 = ops.split_bf16(w, 2, 0)
    wb = w.bfloat16()
    assert torch.equal(w2[:, :K], wb) and torch.equal(w2[:, K:], wb)
    ref = x.double() @ wb.double().t() + b.double()
    y = ops.linear_x2(x, w2, b)
    e2 = _rel64(y, ref)
    e1 = _rel64(ops.linear(hi, wb, b), ref)
    assert e2 < 2e-5 and e2 < e1 / 50, (e2, e1)
    zt = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    hb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    h = ops.linear_x2(x, w2, b, act=_lib.ACT_GELU, pre_out=zt, out_bf16_copy=hb, drop_p=0.1, seed=5)
    idx = (np.arange(M)[:, None] * N + np.arange(N)[None, :]).astype(np.uint64)
    dmask = torch.from_numpy(drop_scale(5, idx, 0.1)).to(DEV).double()
    assert _rel64(h, F.gelu(ref) * dmask) < 2e-5
    assert torch.equal(hb, h.bfloat16()) and _rel64(zt, ref) < 4e-3
    r = torch.randn(M, N, device=DEV)
    y2 = ops.linear_x2(x, w2, b, residual=r)
    assert _rel64(y2, ref + r.double()) < 2e-5
    # producers writing the split image themselves: GEMM bf16 output + low-half copy (copy_lo),
    # LayerNorm yb + ylo, both into the two halves of one [rows, 2·cols] buffer
    hs = torch.empty(M, 2 * N, device=DEV, dtype=torch.bfloat16)
    ops.linear_x2(x, w2, b, act=_lib.ACT_GELU, drop_p=0.1, seed=5, out=hs[:, :N], out_bf16_copy=hs[:, N:], copy_lo=True)
    assert torch.equal(hs[:, :N], h.bfloat16()) and torch.equal(hs[:, N:], (h - h.bfloat16().float()).bfloat16())
    g, be = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    yl = torch.empty(M, K, device=DEV)
    xs = torch.empty(M, 2 * K, device=DEV, dtype=torch.bfloat16)
    ops.layernorm_fwd(x, g, be, 1e-5, y=yl, yb=xs[:, :K], ylo=xs[:, K:])
    assert torch.equal(xs, ops.split_bf16(yl, 2, 2))


@pytest.mark.parametrize("B,T,H,drop_p,masked", [(3, 64, 12, 0.0, True), (2, 100, 4, 0.1, True), (128, 64, 12, 0.1, False),
                                                 (3, 16, 2, 0.0, "all")])
def test_attention_f32_fwd(ops, B, T, H, drop_p, masked):
    """The fp32 text attention forward against float64 (masked, ragged T past one 64-key chunk,
    dropout, an all-masked sample); its saved bf16 copies + LSE drive the bf16 backward kernel to
    the same gradients as from the bf16 forward."""
    torch.manual_seed(T + H)
    D, W = 64, H * 64
    qkv = torch.randn(B * T, 3 * W, device=DEV) * 0.7
    q, k, v = qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:]
    mask = None
    if masked:
        m = torch.ones(B, T, dtype=torch.int32, device=DEV)
        m[0, T - T // 3:] = 0
        m[1, :5] = 0
        if masked == "all":
            m[2, :] = 0
        mask = m.reshape(-1).contiguous()
    o32 = torch.empty(B * T, W, device=DEV)
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=DEV)
    ops.attention_fwd_f32(q, k, v, B=B, T=T, H=H, o32=o32, lse=lse, o=o, o_lo=olo, key_mask=mask, drop_p=drop_p,
                          seed=3)
    qd, kd, vd = (t.double().view(B, T, H, D) for t in (q, k, v))
    ref = attention_ref(qd, kd, vd, mask.view(B, T) if masked else None, drop_p=drop_p, seed=3)
    assert _rel64(o32.view(B, T, H, D), ref) < 1e-5
    assert torch.equal(o, o32.bfloat16()) and torch.equal(olo, (o32 - o.float()).bfloat16())
    sc = (qd.permute(0, 2, 1, 3) @ kd.permute(0, 2, 1, 3).transpose(-1, -2)) / 8.0
    if masked:
        sc = sc + (1.0 - mask.view(B, T)[:, None, None, :].double()) * torch.finfo(torch.float32).min
    lse_ref = torch.logsumexp(sc, -1).reshape(-1)
    fin = lse_ref.abs() < 1e30
    assert _rel64(lse[fin], lse_ref[fin]) < 1e-6
    # the bf16 backward on the saved copies: same gradients as the torch reference
    qb, kb, vb = q.bfloat16(), k.bfloat16(), v.bfloat16()
    do = torch.randn(B * T, W, device=DEV).bfloat16()
    dq, dk, dv = (torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    delta = torch.empty(B * H * T, device=DEV)
    ops.attention_bwd(qb, kb, vb, o, lse, do, dq, dk, dv, B=B, T=T, H=H, delta=delta, key_mask=mask, drop_p=drop_p,
                      seed=3, o_lo=olo)
    qf, kf, vf = (t.float().view(B, T, H, D).clone().requires_grad_() for t in (qb, kb, vb))
    rf = attention_ref(qf, kf, vf, mask.view(B, T) if masked else None, drop_p=drop_p, seed=3)
    rf.backward(do.float().view(B, T, H, D))
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert rel_err(got.view(B, T, H, D), want) < 1e-2


@pytest.mark.parametrize("B,T,H,drop_p,masked,zero_rows", [(3, 64, 12, 0.0, True, True), (2, 100, 4, 0.1, True, True),
                                                           (64, 64, 12, 0.1, False, True), (3, 16, 2, 0.0, "all", True),
                                                           (3, 130, 2, 0.1, "all", False), (2, 37, 3, 0.0, True, False)])
def test_attention_f32_bwd(ops, B, T, H, drop_p, masked, zero_rows):
    """The precise text backward's attention (ste_attention_bwd_f32) against float64 autograd of the
    same forward: fp32 q/k/v and dO, P recomputed from the saved LSE, delta from O hi + lo, the
    forward's dropout mask; one 64-key chunk, ragged and multi-chunk T (dQ summed over chunks in
    order), an all-masked sample under both conventions (SDPA's zero rows, eager's uniform rows)."""
    torch.manual_seed(T * 3 + H)
    D, W = 64, H * 64
    qkv = torch.randn(B * T, 3 * W, device=DEV) * 0.7
    q, k, v = qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:]
    mask = None
    if masked:
        m = torch.ones(B, T, dtype=torch.int32, device=DEV)
        m[0, T - T // 3:] = 0
        m[1, :5] = 0
        if masked == "all":
            m[2, :] = 0
        mask = m.reshape(-1).contiguous()
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=DEV)
    ops.attention_fwd_f32(q, k, v, B=B, T=T, H=H, o32=None, lse=lse, o=o, o_lo=olo, key_mask=mask, drop_p=drop_p,
                          seed=5, zero_masked_rows=zero_rows)
    do = torch.randn(B * T, W, device=DEV)
    dqkv = torch.full((B * T, 3 * W), float("nan"), device=DEV)
    ops.attention_bwd_f32(q, k, v, o, olo, lse, do, dqkv[:, :W], dqkv[:, W:2 * W], dqkv[:, 2 * W:], B=B, T=T, H=H,
                          key_mask=mask, drop_p=drop_p, seed=5, zero_masked_rows=zero_rows)
    qd, kd, vd = (t.double().view(B, T, H, D).clone().requires_grad_() for t in (q, k, v))
    ref = attention_ref(qd, kd, vd, mask.view(B, T) if masked else None, drop_p=drop_p, seed=5)
    if zero_rows and masked:   # SDPA: a sample whose every key is masked gets zero weights
        ref = ref * (mask.view(B, T).sum(1) > 0).double()[:, None, None, None]
    ref.backward(do.double().view(B, T, H, D))
    errs = {n: _rel64(dqkv[:, i * W:(i + 1) * W].view(B, T, H, D), g)
            for i, (n, g) in enumerate((("dq", qd.grad), ("dk", kd.grad), ("dv", vd.grad)))}
    print(f"attention_bwd_f32 B={B} T={T} H={H} drop={drop_p} masked={masked} zero_rows={zero_rows}: {errs}")
    for n, e in errs.items():
        assert e < 5e-5, (n, e)   # fp32 against float64; delta from O's hi + lo halves (~2^-16)


@pytest.mark.parametrize("T,drop_p,f32", [(70, 0.0, False), (130, 0.1, False), (70, 0.0, True), (130, 0.1, True)])
def test_attention_zero_masked_rows(ops, T, drop_p, f32):
    """zero_masked_rows = 1 (the XLM-R SDPA rule): a sample whose every key is masked gets zero
    output, LSE +inf and zero gradients; the other samples are unaffected.  bf16 forward or the
    fp32 text forward, then the bf16 backward."""
    torch.manual_seed(T)
    B, H, D = 3, 2, 64
    W = H * D
    qkv = torch.randn(B * T, 3 * W, device=DEV) * 0.7
    if not f32:
        qkv = qkv.bfloat16()
    q, k, v = qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:]
    m = torch.ones(B, T, dtype=torch.int32, device=DEV)
    m[0, T - T // 3:] = 0
    m[1, :] = 0                      # every key of sample 1 masked
    mask = m.reshape(-1).contiguous()
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=DEV)
    if f32:
        o32 = torch.empty(B * T, W, device=DEV)
        ops.attention_fwd_f32(q, k, v, B=B, T=T, H=H, o32=o32, lse=lse, o=o, o_lo=olo, key_mask=mask, drop_p=drop_p,
                              seed=5, zero_masked_rows=True)
        assert torch.count_nonzero(o32.view(B, T, W)[1]) == 0
    else:
        ops.attention_fwd(q, k, v, B=B, T=T, H=H, o=o, lse=lse, key_mask=mask, drop_p=drop_p, seed=5, o_lo=olo,
                          zero_masked_rows=True)
    assert torch.count_nonzero(o.view(B, T, W)[1]) == 0 and torch.count_nonzero(olo.view(B, T, W)[1]) == 0
    assert torch.isposinf(lse.view(B, H, T)[1]).all() and torch.isfinite(lse.view(B, H, T)[[0, 2]]).all()
    qb, kb, vb = (t.bfloat16() for t in (q, k, v))
    do = torch.randn(B * T, W, device=DEV).bfloat16()
    dq, dk, dv = (torch.full((B * T, W), 7.0, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    ops.attention_bwd(qb, kb, vb, o, lse, do, dq, dk, dv, B=B, T=T, H=H, delta=torch.empty(B * H * T, device=DEV),
                      key_mask=mask, drop_p=drop_p, seed=5, o_lo=olo)
    # reference: the uniform-fill reference with sample 1 multiplied out (zero output, zero gradients)
    qf, kf, vf = (t.float().view(B, T, H, D).clone().requires_grad_() for t in (qb, kb, vb))
    keep = torch.tensor([1.0, 0.0, 1.0], device=DEV).view(B, 1, 1, 1)
    rf = attention_ref(qf, kf, vf, m, drop_p=drop_p, seed=5) * keep
    assert rel_err(o.float().view(B, T, H, D), rf) < 1e-2
    rf.backward(do.float().view(B, T, H, D))
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert torch.count_nonzero(got.view(B, T, W)[1]) == 0
        assert rel_err(got.view(B, T, H, D), want) < 1e-2


# -------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("cols", [4, 160, 260, 768, 1024])   # 4 / 260: partial column groups of a wave
def test_layernorm_fwd_bwd(ops, cols):
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(cols)
    rows = 333
    x = torch.randn(rows, cols, device=DEV) * 2 + 0.5
    g = torch.randn(cols, device=DEV)
    b = torch.randn(cols, device=DEV)
    rs = (torch.rand(rows, device=DEV) > 0.2).float()
    for act in (_lib.ACT_NONE, _lib.ACT_SWISH):
        y = torch.empty_like(x)
        yb = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
        mean, rstd = ops.layernorm_fwd(x, g, b, 1e-5, y=y, yb=yb, row_scale=rs, act=act)
        xr, gr, br = (t.clone().requires_grad_() for t in (x, g, b))
        ref = F.layer_norm(xr, (cols,), gr, br, 1e-5) * rs[:, None]
        if act == _lib.ACT_SWISH:
            ref = F.silu(ref)
        assert rel_err(y, ref) < 1e-5
        assert rel_err(yb, ref) < 5e-3
        dy = torch.randn_like(x)
        ref.backward(dy)
        dres = torch.randn_like(x)
        dx = torch.empty_like(x)
        dxb = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
        dg = torch.zeros(cols, device=DEV)
        db = torch.zeros(cols, device=DEV)
        ops.layernorm_bwd(dy, x, mean, rstd, g, beta=b, dx=dx, dxb=dxb, dres=dres, dgamma=dg, dbeta=db, row_scale=rs,
                          act=act, out_scale=0.5)
        assert rel_err(dx, xr.grad + dres) < 1e-5
        assert rel_err(dxb, 0.5 * (xr.grad + dres)) < 5e-3
        assert rel_err(dg, gr.grad) < 1e-5
        assert rel_err(db, br.grad) < 1e-5


@pytest.mark.parametrize("cols", [1028, 2048])
def test_layernorm_fwd_wide_rows(ops, cols):
    """The forward's widest form (ste_layernorm_fwd admits up to 2,048 columns; the backward 1,024)."""
    torch.manual_seed(cols)
    rows = 129
    x = (torch.randn(rows, cols, device=DEV) * 3 - 1).bfloat16()
    g, b = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV)
    y = torch.empty(rows, cols, device=DEV)
    mean, rstd = ops.layernorm_fwd(x, g, b, 1e-5, y=y)
    xd = x.double()
    assert rel_err(y, F.layer_norm(xd, (cols,), g.double(), b.double(), 1e-5)) < 1e-5
    assert rel_err(mean, xd.mean(1)) < 1e-6
    assert rel_err(rstd, (xd.var(1, unbiased=False) + 1e-5).rsqrt()) < 1e-5


@pytest.mark.parametrize("reduce", [False, True])
def test_layernorm_many_rows_per_wave(ops, reduce):
    """c2-like row counts: each wave walks several rows, the forward and the column-sum-free
    backward with the next row's operands in flight (the prefetch paths); bf16 dy as in the step."""
    torch.manual_seed(11)
    rows, cols = 9001, 1024
    x = torch.randn(rows, cols, device=DEV) * 2 + 0.5
    g, b = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV)
    yb = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
    mean, rstd = ops.layernorm_fwd(x, g, b, 1e-5, yb=yb)
    xr, gr, br = (t.clone().requires_grad_() for t in (x, g, b))
    ref = F.layer_norm(xr, (cols,), gr, br, 1e-5)
    assert rel_err(yb, ref) < 5e-3
    assert torch.allclose(mean, x.mean(1), atol=1e-5)
    dy = torch.randn(rows, cols, device=DEV).bfloat16()
    ref.backward(dy.float())
    dres = torch.randn_like(x)
    dx = torch.empty_like(x)
    dxb = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
    dg = torch.zeros(cols, device=DEV) if reduce else None
    db = torch.zeros(cols, device=DEV) if reduce else None
    ops.layernorm_bwd(dy, x, mean, rstd, g, beta=b, dx=dx, dxb=dxb, dres=dres, dgamma=dg, dbeta=db)
    assert rel_err(dx, xr.grad + dres) < 1e-5
    assert rel_err(dxb, xr.grad + dres) < 5e-3
    if reduce:
        assert rel_err(dg, gr.grad) < 1e-5
        assert rel_err(db, br.grad) < 1e-5


@pytest.mark.parametrize("pair", [False, True])
def test_layernorm_colsums_deterministic(ops, pair):
    """Column sums (dgamma, dbeta, dsum) through the per-block workspace are run-to-run identical
    (fixed-order block sum) and add into the outputs like the atomic path (+=), which they match to
    fp32 rounding; single and chained-pair backward, c2-sized rows."""
    torch.manual_seed(5)
    rows, cols = 31936 // 4, 1024
    x = torch.randn(rows, cols, device=DEV) * 1.5 + 0.3
    g1, b1, g2, b2 = (torch.randn(cols, device=DEV) for _ in range(4))
    y1 = torch.empty(rows, cols, device=DEV)
    (ma, ra), (mb, rb) = ops.layernorm_fwd_pair(dict(x=x, gamma=g1, beta=b1, eps=1e-5, y=y1),
                                                dict(gamma=g2, beta=b2, eps=1e-5,
                                                     yb=torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)))
    dy = torch.randn(rows, cols, device=DEV).bfloat16()
    dres = torch.randn(rows, cols, device=DEV)

    def run():
        sums = [torch.full((cols,), 0.25, device=DEV) for _ in range(5)]   # += onto a non-zero start
        dxb = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
        if pair:
            ops.layernorm_bwd_pair(dict(x=x, mean=ma, rstd=ra, gamma=g1, beta=b1, dxb=dxb, dgamma=sums[0],
                                        dbeta=sums[1], dsum=sums[2]),
                                   dict(dy=dy, x=y1, mean=mb, rstd=rb, gamma=g2, beta=b2, dres=dres, dgamma=sums[3],
                                        dbeta=sums[4]))
        else:
            ops.layernorm_bwd(dy, y1, mb, rb, g2, beta=b2, dres=dres, dxb=dxb, dgamma=sums[3], dbeta=sums[4],
                              dsum=sums[2])
            sums = sums[2:]
        return sums

    first, second = run(), run()
    for a_, b_ in zip(first, second):
        assert torch.equal(a_, b_)
    ops.LN_ATOMIC_COLSUMS = True
    try:
        atomic = run()
    finally:
        ops.LN_ATOMIC_COLSUMS = False
    for a_, b_ in zip(first, atomic):
        assert rel_err(a_, b_) < 1e-5


@pytest.mark.parametrize("case", ["noreduce", "reduce", "frozen_second"])
def test_layernorm_pair_matches_single_calls(ops, case):
    """ste_layernorm_fwd_pair / _bwd_pair (a Conformer layer's final LN chained with the next
    layer's FFN1 LN) against the same two LayerNorms run as single calls: forward outputs (fp32,
    bf16, the second LN's MX-fp8 copy) bit for bit; input gradients to fp32 rounding (the pair keeps
    the intermediate gradient in registers and sums its row terms in another order than the
    chained calls, which round it to an fp32 tensor in between), column sums to atomic-order
    rounding.  noreduce: no column sums (the residual row preloaded); reduce: both
    LNs trainable; frozen_second: the later LN frozen (null dgamma/dbeta) under a trainable first."""
    torch.manual_seed(12)
    rows, cols = 5003, 1024
    x = torch.randn(rows, cols, device=DEV) * 1.5 + 0.3
    g1, b1 = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV) * 0.1
    g2, b2 = torch.randn(cols, device=DEV), torch.randn(cols, device=DEV) * 0.1
    E = lambda dt=torch.float32: torch.empty(rows, cols, device=DEV, dtype=dt)  # noqa: E731
    q8 = lambda: (E(torch.uint8), torch.empty(rows, cols // 32, device=DEV, dtype=torch.uint8))  # noqa: E731
    # forward: pair vs singles
    y1, y1b, y2b, q2 = E(), E(torch.bfloat16), E(torch.bfloat16), q8()
    (ma, ra), (mb, rb) = ops.layernorm_fwd_pair(dict(x=x, gamma=g1, beta=b1, eps=1e-5, y=y1, yb=y1b),
                                                dict(gamma=g2, beta=b2, eps=1e-5, yb=y2b, q8=q2))
    y1s, y1bs, y2bs, q2s = E(), E(torch.bfloat16), E(torch.bfloat16), q8()
    mas, ras = ops.layernorm_fwd(x, g1, b1, 1e-5, y=y1s, yb=y1bs)
    mbs, rbs = ops.layernorm_fwd(y1s, g2, b2, 1e-5, yb=y2bs, q8=q2s)
    for got, want in ((y1, y1s), (y1b, y1bs), (y2b, y2bs), (q2[0], q2s[0]), (q2[1], q2s[1]), (ma, mas), (ra, ras),
                      (mb, mbs), (rb, rbs)):
        assert torch.equal(got, want)
    # backward: b (the later LN, with dy and the residual gradient) then a, fused vs chained
    dy2 = torch.randn(rows, cols, device=DEV).bfloat16()
    dres = torch.randn(rows, cols, device=DEV)
    tr_a = case != "noreduce"
    tr_b = case == "reduce"
    Z = lambda on: torch.zeros(cols, device=DEV) if on else None  # noqa: E731
    dga, dba, dsa, dgb, dbb = Z(tr_a), Z(tr_a), Z(tr_a), Z(tr_b), Z(tr_b)
    dxa, dxab = E(), E(torch.bfloat16)
    ops.layernorm_bwd_pair(
        dict(x=x, mean=ma, rstd=ra, gamma=g1, beta=b1, dx=dxa, dxb=dxab, out_scale=0.5, dgamma=dga, dbeta=dba,
             dsum=dsa),
        dict(dy=dy2, x=y1, mean=mb, rstd=rb, gamma=g2, beta=b2, dres=dres, dgamma=dgb, dbeta=dbb))
    dmid = E()
    dgbs, dbbs, dgas, dbas, dsas = Z(tr_b), Z(tr_b), Z(tr_a), Z(tr_a), Z(tr_a)
    ops.layernorm_bwd(dy2, y1s, mbs, rbs, g2, beta=b2, dres=dres, dx=dmid, dgamma=dgbs, dbeta=dbbs)
    dxas, dxabs = E(), E(torch.bfloat16)
    ops.layernorm_bwd(dmid, x, mas, ras, g1, beta=b1, dx=dxas, dxb=dxabs, out_scale=0.5, dgamma=dgas, dbeta=dbas,
                      dsum=dsas)
    print(f"LN pair bwd [{case}]: dx {rel_err(dxa, dxas):.2e}, dxb {rel_err(dxab.float(), dxabs.float()):.2e}")
    assert rel_err(dxa, dxas) < 1e-6
    assert rel_err(dxab.float(), dxabs.float()) < 1e-4      # bf16 copies: the odd element one ulp apart
    for got, want in ((dga, dgas), (dba, dbas), (dsa, dsas), (dgb, dgbs), (dbb, dbbs)):
        if want is not None:
            assert rel_err(got, want) < 1e-5


# -------------------------------------------------------------- attention
def _attn_case(ops, B, T, H, rel, masked, drop_p, seed=7, qk_scale=0.7, v_common=0.0, o_lo=False, tol=1e-2, left=64,
               right=8):
    """left/right: the relative-distance window (w2v-bert: 64 / 8; nrel = left + right + 1 bins).
    v_common > 0: every value row is a shared per-(batch, head) vector plus 0.05 noise, and
    qk_scale small makes the attention near-uniform (the random-init encoder regime): O ≈ mean(V)
    and dS = P(dP - delta) is a small difference of large terms."""
    torch.manual_seed(T * 7 + H)
    D = 64
    W = H * D
    qkv = torch.randn(B * T, 3 * W, device=DEV) * qk_scale
    if v_common:
        common = torch.randn(B, 1, W, device=DEV) * v_common
        qkv[:, 2 * W:] = (common + 0.05 * torch.randn(B, T, W, device=DEV)).reshape(B * T, W)
    qkv = qkv.bfloat16()
    q, k, v = qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:]
    mask = None
    if masked:
        m = torch.ones(B, T, dtype=torch.int32, device=DEV)
        m[0, T - T // 3:] = 0
        if B > 1:
            m[1, :5] = 0
        if masked == "all" and B > 2:
            m[2, :] = 0          # every key masked: uniform attention, like the reference's finfo.min fill
        mask = m.reshape(-1).contiguous()
    nrel = left + right + 1
    E = (torch.randn(nrel, D, device=DEV) * 0.5).bfloat16() if rel else None
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o) if o_lo else None
    lse = torch.empty(B * H * T, device=DEV)
    ops.attention_fwd(q, k, v, B=B, T=T, H=H, o=o, lse=lse, key_mask=mask, rel_E=E, rel_left=left, rel_right=right,
                      drop_p=drop_p, seed=seed, o_lo=olo)
    qf, kf, vf = (t.float().view(B, T, H, D).clone().requires_grad_() for t in (q, k, v))
    Ef = E.float().clone().requires_grad_() if rel else None
    ref = attention_ref(qf, kf, vf, mask.view(B, T) if masked else None, Ef, left=left, right=right, drop_p=drop_p,
                        seed=seed)
    assert rel_err(o.view(B, T, H, D), ref) < 1e-2
    with torch.no_grad():  # saved log-sum-exp of the scaled, biased, masked scores
        qh, kh = qf.permute(0, 2, 1, 3), kf.permute(0, 2, 1, 3)
        sc = qh @ kh.transpose(-1, -2)
        if rel:
            pos = torch.arange(T, device=DEV)
            dist = (pos.view(1, -1) - pos.view(-1, 1)).clamp(-left, right) + left
            sc = sc + torch.gather(qh @ Ef.t(), 3, dist.view(1, 1, T, T).expand(B, H, T, T))
        sc = sc / math.sqrt(D)
        if masked:
            sc = sc + (1.0 - mask.view(B, T)[:, None, None, :].float()) * torch.finfo(torch.float32).min
        lse_ref = torch.logsumexp(sc, -1).reshape(-1)
        fin = lse_ref.abs() < 1e30
        assert rel_err(lse[fin], lse_ref[fin]) < 1e-3
    do = torch.randn(B * T, W, device=DEV).bfloat16()
    ref.backward(do.float().view(B, T, H, D))
    dqkv = torch.zeros(B * T, 3 * W, device=DEV, dtype=torch.bfloat16)
    delta = torch.empty(B * H * T, device=DEV)
    dE = torch.zeros(nrel, D, device=DEV) if rel else None
    gw = torch.empty(B * H * T * 80, device=DEV) if rel else None
    ops.attention_bwd(q, k, v, o, lse, do, dqkv[:, :W], dqkv[:, W:2 * W], dqkv[:, 2 * W:], B=B, T=T, H=H, delta=delta,
                      key_mask=mask, rel_E=E, rel_left=left, rel_right=right, drop_p=drop_p, seed=seed, dE=dE,
                      gwork=gw, o_lo=olo)
    errs = {"dq": rel_err(dqkv[:, :W].view(B, T, H, D), qf.grad), "dk": rel_err(dqkv[:, W:2 * W].view(B, T, H, D), kf.grad),
            "dv": rel_err(dqkv[:, 2 * W:].view(B, T, H, D), vf.grad)}
    if rel:
        errs["dE"] = rel_err(dE, Ef.grad)
    if o_lo:
        if not drop_p:
            # ~fp32 output: the saving forward weights V by hi + lo P (~2^-16 of p)
            assert rel_err(o.float() + olo.float(), ref.reshape(B * T, W)) < 1e-4
    print(f"attention B={B} T={T} H={H} rel={rel} v_common={v_common} o_lo={o_lo}: {errs}")
    for k_, e in errs.items():
        assert e < tol, (k_, e)
    return errs


@pytest.mark.parametrize("T", [17, 40, 99, 150, 499])   # T < 64: the small-T dE kernel; else the MFMA one
def test_attention_relkey(ops, T):
    _attn_case(ops, B=2, T=T, H=2, rel=True, masked=True, drop_p=0.0)


@pytest.mark.parametrize("T", [40, 130])
def test_attention_relkey_dE_deterministic(ops, T):
    """The MFMA dE kernel (T >= 64) writes one partial per (batch, head) and sums them in a fixed
    order; the small-T kernel walks every (batch, head) and row in order, one block per 16 bins:
    two identical backward calls give bit-identical dE (16 partials here, > one 16-way lane group)."""
    B, H, D = 4, 4, 64
    W = H * D
    torch.manual_seed(7)
    qkv = (torch.randn(B * T, 3 * W, device=DEV) * 0.5).bfloat16()
    q, k, v = qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:]
    E = (torch.randn(73, D, device=DEV) * 0.5).bfloat16()
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=DEV)
    ops.attention_fwd(q, k, v, B=B, T=T, H=H, o=o, lse=lse, rel_E=E, o_lo=olo)
    do = torch.randn(B * T, W, device=DEV).bfloat16()
    outs = []
    for _ in range(2):
        dqkv = torch.zeros(B * T, 3 * W, device=DEV, dtype=torch.bfloat16)
        dE = torch.zeros(73, D, device=DEV)
        ops.attention_bwd(q, k, v, o, lse, do, dqkv[:, :W], dqkv[:, W:2 * W], dqkv[:, 2 * W:], B=B, T=T, H=H,
                          delta=torch.empty(B * H * T, device=DEV), rel_E=E, dE=dE,
                          gwork=torch.empty(B * H * T * 80, device=DEV), o_lo=olo)
        outs.append(dE)
    assert torch.equal(outs[0], outs[1])
    assert outs[0].abs().sum() > 0


def test_attention_relkey_fully_masked_row(ops):
    _attn_case(ops, B=3, T=130, H=2, rel=True, masked="all", drop_p=0.0)


def test_attention_relkey_unmasked_long(ops):
    _attn_case(ops, B=1, T=700, H=1, rel=True, masked=False, drop_p=0.0)


def test_attention_relkey_near_uniform_delta_precision(ops):
    """Random-init regime (near-uniform attention, values with a large shared component): the
    backward's delta = rowsum(dO·O) must come from the ~fp32 output (o_lo) — from the bf16-stored
    O alone the dQ/dK/dE errors are several times larger (both measured and printed)."""
    kw = dict(B=2, T=499, H=2, rel=True, masked=True, drop_p=0.0, qk_scale=0.3, v_common=1.0)
    coarse = _attn_case(ops, **kw, o_lo=False, tol=1.0)
    fine = _attn_case(ops, **kw, o_lo=True, tol=1e-2)
    assert fine["dq"] <= coarse["dq"] and fine["dk"] <= coarse["dk"]


@pytest.mark.parametrize("T", [499, 1499])
def test_attention_relkey_o_lo(ops, T):
    """The o_lo path at the c2 and c5 (30 s) frame counts, masked."""
    _attn_case(ops, B=2, T=T, H=2, rel=True, masked=True, drop_p=0.0, o_lo=True, tol=1e-2)


@pytest.mark.parametrize("T,left,right", [(499, 64, 8), (1499, 64, 8), (300, 71, 8), (4200, 64, 8)])
def test_attention_relkey_o_lo_common_value(ops, T, left, right):
    """What the backward's delta = dO·(O + O_lo) relies on: when every value row of a (batch, head)
    is the same vector c, O + O_lo must be c to the split's ~16 bits whatever the weights, so
    that dP - delta cancels the common component exactly (the forward's weights sum to 1: the row
    sum is taken over the same rounded P the PV product uses).  Masked, at the c2 / c5 frame
    counts, the widest window (rel2 forward) and past the rel4 forward's key-tile limit."""
    torch.manual_seed(T)
    B, H, D = 2, 2, 64
    W = H * D
    q = (torch.randn(B * T, W, device=DEV) * 0.7).bfloat16()
    k = (torch.randn(B * T, W, device=DEV) * 0.7).bfloat16()
    c = torch.randn(B, 1, W, device=DEV).bfloat16()
    v = c.expand(B, T, W).reshape(B * T, W).contiguous()
    m = torch.ones(B, T, dtype=torch.int32, device=DEV)
    m[0, T - T // 3:] = 0
    m[1, :5] = 0
    E = (torch.randn(left + right + 1, D, device=DEV) * 0.5).bfloat16()
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=DEV)
    ops.attention_fwd(q, k, v, B=B, T=T, H=H, o=o, lse=lse, key_mask=m.reshape(-1).contiguous(), rel_E=E,
                      rel_left=left, rel_right=right, o_lo=olo)
    full = (o.float() + olo.float()).view(B, T, W)
    err = ((full - c.float()).abs().max() / c.float().abs().max()).item()
    print(f"common-value O + O_lo, T={T} window {left}/{right}: max rel {err:.2e}")
    assert err < 3e-5   # hi + lo bf16 carry ~16 mantissa bits of the fp32 O (2^-16 = 1.5e-5)


@pytest.mark.parametrize("left,right", [(16, 16), (74, 0), (68, 8), (71, 8)])
def test_attention_relkey_window(ops, left, right):
    """Other relative windows through the C ABI (nrel = 33, 75, 77, 80): 33 and 75 on the v4 forward
    (at most 75 bins), 77 and 80 (the table capacity) on the v2 forward; all on the v3 backward, with
    and without the hi/lo split."""
    for o_lo in (False, True):
        _attn_case(ops, B=2, T=300, H=2, rel=True, masked=True, drop_p=0.0, o_lo=o_lo, left=left, right=right)


@pytest.mark.parametrize("T", [99, 300])
def test_attention_relkey_dropout(ops, T):
    """Relative keys with attention dropout (the generic forward / dQ / dK-dV kernels; the
    w2v-bert configs run the audio attention without dropout), standard and widest window."""
    _attn_case(ops, B=2, T=T, H=2, rel=True, masked=True, drop_p=0.1)
    _attn_case(ops, B=2, T=T, H=2, rel=True, masked=True, drop_p=0.1, left=71, right=8)


@pytest.mark.parametrize("o_lo", [False, True])
def test_attention_relkey_past_v4_limit(ops, o_lo):
    """T = 4,200 frames (84 s of audio) is past the v4 forward's 64 key tiles (rel4::MAXT): the v2
    forward runs (with and without the hi/lo split), then the v3 backward, masked."""
    _attn_case(ops, B=1, T=4200, H=1, rel=True, masked=True, drop_p=0.0, o_lo=o_lo)


@pytest.mark.parametrize("drop_p", [0.0, 0.1])
def test_attention_text_o_lo(ops, drop_p):
    _attn_case(ops, B=3, T=64, H=3, rel=False, masked=True, drop_p=drop_p, o_lo=True, qk_scale=0.3, v_common=1.0,
               tol=1e-2)


@pytest.mark.parametrize("T", [37, 130])
def test_attention_text_ragged(ops, T):
    """Text attention at a partial key tile and past two tiles, with dropout."""
    _attn_case(ops, B=3, T=T, H=3, rel=False, masked=True, drop_p=0.1)


@pytest.mark.parametrize("drop_p", [0.0, 0.1])
def test_attention_text(ops, drop_p):
    _attn_case(ops, B=3, T=64, H=3, rel=False, masked=True, drop_p=drop_p)


# ---------------------------------------------------------------- conv
@pytest.mark.parametrize("T,Cc", [(37, 128), (150, 128), (37, 256), (499, 512), (300, 1024), (1499, 128)])
def test_glu_dwconv(ops, T, Cc):
    torch.manual_seed(T)
    B = 2
    pre = torch.randn(B * T, 2 * Cc, device=DEV).bfloat16()
    w = torch.randn(Cc, 31, device=DEV) * 0.2
    out = torch.empty(B * T, Cc, device=DEV, dtype=torch.bfloat16)
    ops.glu_dwconv_fwd(pre, w, out, B, T)
    pr = pre.float().clone().requires_grad_()
    wr = w.clone().requires_grad_()
    ref = glu_dwconv_ref(pr, wr, B, T)
    assert rel_err(out, ref) < 5e-3
    do = torch.randn(B * T, Cc, device=DEV).bfloat16()
    ref.backward(do.float())
    dpre = torch.empty_like(pre)
    dw = torch.zeros_like(w)
    ops.glu_dwconv_bwd(pre, w, do, dpre, dw, B, T)
    assert rel_err(dpre, pr.grad) < 5e-3
    assert rel_err(dw, wr.grad) < 1e-4


# ---------------------------------------------------------------- fbank
def test_fbank_matches_golden(ops):
    from conftest import GOLDEN
    z = np.load(GOLDEN / "fbank_golden.npz")
    cases = list(z["cases"])
    waves = [z[f"{c}_wave"] for c in cases]
    N = max(w.size for w in waves)
    wav = torch.zeros(len(waves), N, device=DEV)
    for i, w in enumerate(waves):
        wav[i, : w.size] = torch.from_numpy(w)
    lens = torch.tensor([w.size for w in waves], dtype=torch.int32, device=DEV)
    Tmax = z["batch_feats"].shape[1]
    feats, mask = ops.fbank(wav, lens, Tmax, pad_value=1.0, mask_mode=0)
    np.testing.assert_array_equal(mask.cpu().numpy(), z["batch_mask"])
    np.testing.assert_allclose(feats.cpu().numpy(), z["batch_feats"], atol=FBANK_ATOL, rtol=0)
    feats1, mask1 = ops.fbank(wav, lens, Tmax, pad_value=1.0, mask_mode=1)
    for i, c in enumerate(cases):
        T = z[f"{c}_feats"].shape[0]
        np.testing.assert_array_equal(mask1[i, :T].cpu().numpy(), z[f"{c}_mask"])


FBANK_ATOL = 5e-4   # half the SURVEY §8(d) fp32 bound (1e-3) on CMVN-normalised features; measured <= 3.8e-4


_FBANK_THREADS = r"""
import sys, threading, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from speech_transcript_embeddings_amd import ops
z = np.load(sys.argv[2])
cases = list(z["cases"])
waves = [z[f"{c}_wave"] for c in cases]
N = max(w.size for w in waves)
wav = torch.zeros(len(waves), N, device="cuda")
for i, w in enumerate(waves):
    wav[i, : w.size] = torch.from_numpy(w)
lens = torch.tensor([w.size for w in waves], dtype=torch.int32, device="cuda")
Tmax = z["batch_feats"].shape[1]
out, barrier = {}, threading.Barrier(2)

def run(k):
    s = torch.cuda.Stream()
    barrier.wait()                      # both threads enter the library's first call together
    with torch.cuda.stream(s):
        f, m = ops.fbank(wav, lens, Tmax, pad_value=1.0, mask_mode=0)
    s.synchronize()
    out[k] = (f.cpu().numpy(), m.cpu().numpy())

ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
[t.start() for t in ts]
[t.join() for t in ts]
for k in range(2):
    np.testing.assert_array_equal(out[k][1], z["batch_mask"])
    np.testing.assert_allclose(out[k][0], z["batch_feats"], atol=float(sys.argv[3]), rtol=0)
assert np.array_equal(out[0][0], out[1][0])
print("fbank-threads-ok")
"""


def test_fbank_first_calls_concurrent_on_two_streams():
    """ste_fbank keeps no lazily built device state.  In a fresh process (fresh device
    context), two threads make the library's first fbank calls at the same moment on two streams;
    both match the reference's golden features."""
    import subprocess
    import sys
    from conftest import GOLDEN, ROOT
    r = subprocess.run([sys.executable, "-c", _FBANK_THREADS, str(ROOT), str(GOLDEN / "fbank_golden.npz"),
                        str(FBANK_ATOL)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "fbank-threads-ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_fbank_config_size_clips_match_reference_extractor(ops):
    """BASELINE clip lengths and edge paths against the reference extractor
    (tests/golden/fbank_golden_long.npz, made by make_golden.py --fbank-long): a c2 10 s clip, a
    c5 30 s clip, an odd frame count (one padded frame), 2 s of zeros inside a loud (x8, > 1.0)
    clip, and an all-silent clip — per clip with the extractor's mask semantics, and batched
    (ragged, padded to 30 s) with the reference collate's mask."""
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, str(GOLDEN))
    from fbank_cases import LONG_CASES, long_case_wave
    z = np.load(GOLDEN / "fbank_golden_long.npz")
    waves = [long_case_wave(c) for c, _, _ in LONG_CASES]
    N = max(w.size for w in waves)
    wav = torch.zeros(len(waves), N, device=DEV)
    for i, w in enumerate(waves):
        wav[i, : w.size] = torch.from_numpy(w)
    lens = torch.tensor([w.size for w in waves], dtype=torch.int32, device=DEV)
    Tmax = z["batch_mask"].shape[1]
    feats1, mask1 = ops.fbank(wav, lens, Tmax, pad_value=1.0, mask_mode=1)
    feats0, mask0 = ops.fbank(wav, lens, Tmax, pad_value=1.0, mask_mode=0)
    np.testing.assert_array_equal(mask0.cpu().numpy(), z["batch_mask"])
    errs = {}
    for i, (c, _, _) in enumerate(LONG_CASES):
        ref = z[f"{c}_feats"]
        T = ref.shape[0]
        got = feats1[i, :T].cpu().numpy()
        errs[c] = float(np.abs(got - ref).max())
        np.testing.assert_array_equal(mask1[i, :T].cpu().numpy(), z[f"{c}_mask"])
        assert torch.equal(feats0[i, :T], feats1[i, :T])
    print("fbank max abs error vs reference extractor:", errs)
    for c, e in errs.items():
        assert e <= FBANK_ATOL, (c, e)


def test_fbank_bin_group_paths_agree(ops):
    """The fused statistics + normalise kernel picks its bin group (16, 8, 4, 2 mel bins per block)
    from the batch's frame capacity 2·Tmax, and past 2-bin columns of 64 KB falls back to the
    separate statistics and normalise kernels.  A padded Tmax drives the same clips through every
    path: identical features (bit for bit: the same frame-ordered sums and IEEE divisions), the
    padding rows of each mask mode, and the masks."""
    torch.manual_seed(3)
    lens = [160000, 123457, 48000, 400, 399]   # 10 s, ragged, 3 s, one frame, no frame
    N = max(lens)
    wav = torch.randn(len(lens), N, device=DEV) * 0.1
    for i, n in enumerate(lens):
        wav[i, n:] = 0
    lt = torch.tensor(lens, dtype=torch.int32, device=DEV)
    T0 = 499
    for mode in (0, 1):
        base, bmask = ops.fbank(wav, lt, T0, pad_value=1.0, mask_mode=mode)
        # Tmax -> Fp = 2 Tmax: 16 bins (T0), 8 (1,500), 4 (3,000), 2 (6,000), fallback (17,000)
        for T in (1500, 3000, 6000, 17000):
            f, m = ops.fbank(wav, lt, T, pad_value=1.0, mask_mode=mode)
            assert torch.equal(f[:, :T0], base), (mode, T)
            assert torch.equal(m[:, :T0], bmask), (mode, T)
            assert not m[:, T0:].any()
            assert bool((f[:, T0:] == (0.0 if mode == 0 else 1.0)).all()), (mode, T)


def test_feature_extractor_api():
    """Drop-in extractor (ref:856-866 call shape) per clip and batched vs the real extractor's output."""
    from conftest import GOLDEN
    from speech_transcript_embeddings_amd.features import SeamlessM4TFeatureExtractor, fbank
    z = np.load(GOLDEN / "fbank_golden.npz")
    fe = SeamlessM4TFeatureExtractor(padding_value=1.0)
    cases = list(z["cases"])
    for c in cases:
        out = fe(z[f"{c}_wave"], sampling_rate=16000, return_tensors="pt")
        T = z[f"{c}_feats"].shape[0]
        assert out["input_features"].shape == (1, T, 160) and out["attention_mask"].shape == (1, T)
        np.testing.assert_allclose(out["input_features"][0].cpu().numpy(), z[f"{c}_feats"], atol=FBANK_ATOL, rtol=0)
        np.testing.assert_array_equal(out["attention_mask"][0].cpu().numpy(), z[f"{c}_mask"])
    with pytest.raises(ValueError):
        fe(z[f"{cases[0]}_wave"], sampling_rate=8000)
    # batched call pads to the longest clip with padding_value, mask 0 there
    outb = fe([z[f"{c}_wave"] for c in cases], sampling_rate=16000)
    for i, c in enumerate(cases):
        T = z[f"{c}_feats"].shape[0]
        np.testing.assert_allclose(outb["input_features"][i, :T].cpu().numpy(), z[f"{c}_feats"], atol=FBANK_ATOL, rtol=0)
        assert outb["input_features"][i, T:].eq(1.0).all() and outb["attention_mask"][i, T:].eq(0).all()
    # training-path variant: collate semantics
    N = max(z[f"{c}_wave"].size for c in cases)
    wav = torch.zeros(len(cases), N, device=DEV)
    for i, c in enumerate(cases):
        wav[i, : z[f"{c}_wave"].size] = torch.from_numpy(z[f"{c}_wave"])
    lens = torch.tensor([z[f"{c}_wave"].size for c in cases], dtype=torch.int32)
    feats, mask = fbank(wav, lens)
    np.testing.assert_array_equal(mask.cpu().numpy(), z["batch_mask"])
    np.testing.assert_allclose(feats.cpu().numpy(), z["batch_feats"], atol=FBANK_ATOL, rtol=0)


# ---------------------------------------------------------------- heads
@pytest.mark.parametrize("B,L,H,Hh", [(3, 50, 256, 128), (3, 64, 768, 384), (2, 499, 1024, 512),
                                      (64, 499, 1024, 512)])
def test_attn_pool(ops, B, L, H, Hh):
    """Score/softmax/weighted-sum forward and the four-launch backward at a small case, the text
    head's shape (Hh=384: ragged thread groups), the audio head's (L=499: partial row chunks) and
    the c2 audio batch (64-row chunks instead of 16)."""
    torch.manual_seed(3)
    h = torch.randn(B * L, H, device=DEV).bfloat16()
    t = torch.tanh(torch.randn(B * L, Hh, device=DEV)).bfloat16()
    w2 = torch.randn(Hh, device=DEV) * 0.3
    b2 = torch.randn(1, device=DEV)
    mask = torch.ones(B * L, dtype=torch.int32, device=DEV)
    mask[L - 7:L] = 0
    if B > 2:   # ragged lengths (1 .. L) and one all-masked sample (uniform weights, as the -1e9 fill gives)
        lens = torch.randint(1, L + 1, (B,), generator=torch.Generator().manual_seed(L))
        lens[1] = 0
        mask = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int32).reshape(-1).to(DEV)
    weights = torch.empty(B * L, device=DEV)
    pooled = torch.empty(B, H, device=DEV)
    ops.attn_pool_fwd(t, w2, b2, h, mask, B, L, weights, pooled)
    if B > 2:
        assert torch.allclose(weights.view(B, L)[1], torch.full((L,), 1.0 / L, device=DEV))
    tr = t.float().clone().requires_grad_()
    hr = h.float().clone().requires_grad_()
    w2r = w2.clone().requires_grad_()
    b2r = b2.clone().requires_grad_()
    s = (tr @ w2r + b2r).view(B, L).masked_fill(mask.view(B, L) == 0, -1e9)
    wref = torch.softmax(s, 1)
    pref = torch.bmm(wref.unsqueeze(1), hr.view(B, L, H)).squeeze(1)
    assert rel_err(pooled, pref) < 1e-5
    dp = torch.randn(B, H, device=DEV)
    pref.backward(dp)
    dh = torch.zeros(B * L, H, device=DEV)
    dz = torch.empty(B * L, Hh, device=DEV, dtype=torch.bfloat16)
    dw2 = torch.full((Hh,), 0.5, device=DEV)      # accumulated into (+=)
    db2 = torch.zeros(1, device=DEV)
    db1 = torch.zeros(Hh, device=DEV)
    dz_lo = torch.empty_like(dz)
    ops.attn_pool_bwd(t, w2, h, weights, dp, B, L, dh, dz, dw2, db2, db1=db1, dz_lo=dz_lo, mask=mask)
    dz_ref = tr.grad * (1 - t.float() ** 2)
    assert rel_err(dh, hr.grad) < 1e-5
    assert rel_err(dz, dz_ref) < 5e-3
    assert rel_err(dz.float() + dz_lo.float(), dz_ref) < 2e-5   # hi + lo: ~fp32
    assert rel_err(db1, dz_ref.sum(0)) < 1e-5                   # fp32 column sums (Σ dscore = 0 cancellation)
    assert rel_err(dw2 - 0.5, w2r.grad) < 1e-4
    db1_again = torch.zeros(Hh, device=DEV)                     # column sums without atomics: bitwise repeatable
    ops.attn_pool_bwd(t, w2, h, weights, dp, B, L, torch.zeros_like(dh), dz, None, None, db1=db1_again, mask=mask)
    assert torch.equal(db1_again, db1)
    assert abs(db2.item() - b2r.grad.item()) < 1e-4


@pytest.mark.parametrize("B,L,H,Hh", [(3, 64, 768, 384), (128, 64, 768, 384)])
def test_attn_pool_f32(ops, B, L, H, Hh):
    """The text side's fp32 pooling (fp32 scorer activations and states, fp32 dz) against
    float64, including ragged and all-masked samples."""
    torch.manual_seed(7)
    h = torch.randn(B * L, H, device=DEV) + 3.0        # a large common component, as encoder states have
    t = torch.tanh(torch.randn(B * L, Hh, device=DEV))
    w2 = torch.randn(Hh, device=DEV) * 0.3
    b2 = torch.randn(1, device=DEV)
    lens = torch.randint(1, L + 1, (B,), generator=torch.Generator().manual_seed(L))
    lens[1] = 0
    mask = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int32).reshape(-1).to(DEV)
    weights = torch.empty(B * L, device=DEV)
    pooled = torch.empty(B, H, device=DEV)
    ops.attn_pool_fwd_f32(t, w2, b2, h, mask, B, L, weights, pooled)
    tr = t.double().clone().requires_grad_()
    hr = h.double().clone().requires_grad_()
    w2r = w2.double().clone().requires_grad_()
    s = (tr @ w2r + b2.double()).view(B, L).masked_fill(mask.view(B, L) == 0, -1e9)
    pref = torch.bmm(torch.softmax(s, 1).unsqueeze(1), hr.view(B, L, H)).squeeze(1)
    assert _rel64(pooled, pref) < 1e-6
    dp = torch.randn(B, H, device=DEV)
    pref.backward(dp.double())
    dh = torch.zeros(B * L, H, device=DEV)
    dz = torch.empty(B * L, Hh, device=DEV)
    dw2 = torch.zeros(Hh, device=DEV)
    db1 = torch.zeros(Hh, device=DEV)
    ops.attn_pool_bwd_f32(t, w2, h, weights, dp, B, L, dh, dz, dw2, None, db1=db1, mask=mask)
    dz_ref = tr.grad * (1 - t.double() ** 2)
    assert _rel64(dh, hr.grad) < 1e-6
    assert _rel64(dz, dz_ref) < 1e-5
    assert _rel64(db1, dz_ref.sum(0)) < 1e-4
    assert _rel64(dw2, w2r.grad) < 1e-4


@pytest.mark.parametrize("cls", [False, True])
def test_mean_pool(ops, cls):
    """use_attentive_pooling=False: text CLS row (ref:578-580), audio masked mean with
    clamp(sum(mask), 1e-9) (ref:621-636): a ragged row and an all-masked row (pools to 0)."""
    torch.manual_seed(5)
    B, L, H = 4, 37, 1024
    h = torch.randn(B * L, H, device=DEV).bfloat16()
    mask = torch.ones(B, L, dtype=torch.int32, device=DEV)
    mask[1, 20:] = 0
    mask[2] = 0
    weights = torch.empty(B * L, device=DEV)
    pooled = torch.empty(B, H, device=DEV)
    pooledb = torch.empty(B, H, device=DEV, dtype=torch.bfloat16)
    ops.mean_pool_fwd(h, mask, B, L, cls, weights, pooled, pooledb)
    hr = h.float().view(B, L, H).clone().requires_grad_()
    if cls:
        pref = hr[:, 0, :]
    else:
        m = mask.view(B, L, 1).expand(B, L, H).long()
        pref = (hr * m).sum(1) / torch.clamp(m.sum(1), min=1e-9)
    assert rel_err(pooled, pref) < 1e-6
    assert (pooledb.float() - pooled).abs().max().item() <= pooled.abs().max().item() * 2 ** -8
    if not cls:
        assert pooled[2].abs().max().item() == 0.0
    pooled32 = torch.empty(B, H, device=DEV)
    h32 = torch.randn(B * L, H, device=DEV)
    ops.mean_pool_fwd(h32, mask, B, L, cls, torch.empty(B * L, device=DEV), pooled32)   # fp32 states (text side)
    h32r = h32.double().view(B, L, H)
    p32 = h32r[:, 0, :] if cls else (h32r * mask.view(B, L, 1)).sum(1) / torch.clamp(mask.view(B, L, 1).sum(1), min=1e-9)
    assert _rel64(pooled32, p32) < 1e-6
    dp = torch.randn(B, H, device=DEV)
    pref.backward(dp)
    dh = torch.ones(B * L, H, device=DEV)  # += semantics
    ops.weighted_pool_bwd(weights, dp, B, L, dh)
    assert rel_err(dh - 1.0, hr.grad.view(B * L, H)) < 1e-6


@pytest.mark.parametrize("drop_p", [0.0, 0.1])
def test_xattn1(ops, drop_p):
    torch.manual_seed(4)
    B, S, P, nh = 3, 40, 256, 8
    q = torch.randn(B, P, device=DEV)
    kv = torch.randn(B * S, 2 * P, device=DEV).bfloat16()
    k, v = kv[:, :P], kv[:, P:]
    mask = torch.ones(B * S, dtype=torch.int32, device=DEV)
    mask[S - 9:S] = 0
    probs = torch.empty(B * nh * S, device=DEV)
    out = torch.empty(B, P, device=DEV)
    seed = 99
    ops.xattn1_fwd(q, k, v, mask, B, S, nh, probs, out, drop_p=drop_p, seed=seed)
    d = P // nh
    qr = q.clone().requires_grad_()
    kr = k.float().clone().requires_grad_()
    vr = v.float().clone().requires_grad_()
    qh = qr.view(B, 1, nh, d).transpose(1, 2)
    kh = kr.view(B, S, nh, d).transpose(1, 2)
    vh = vr.view(B, S, nh, d).transpose(1, 2)
    a = (qh @ kh.transpose(-2, -1)) * d ** -0.5
    a = a.masked_fill(mask.view(B, 1, 1, S) == 0, -1e9).softmax(-1)
    if drop_p > 0:
        idx = np.arange(B * nh * S).astype(np.uint64)
        a = a * torch.from_numpy(drop_scale(seed, idx, drop_p)).to(DEV).view(B, nh, 1, S)
    ref = (a @ vh).transpose(1, 2).reshape(B, P)
    assert rel_err(out, ref) < 1e-5
    do = torch.randn(B, P, device=DEV)
    ref.backward(do)
    dq = torch.empty(B, P, device=DEV)
    dk = torch.zeros(B * S, P, device=DEV)
    dv = torch.zeros(B * S, P, device=DEV)
    ops.xattn1_bwd(q, k, v, probs, do, B, S, nh, dq, dk, dv, drop_p=drop_p, seed=seed, mask=mask)
    assert rel_err(dq, qr.grad) < 1e-5
    assert rel_err(dk, kr.grad) < 1e-5
    assert rel_err(dv, vr.grad) < 1e-5


@pytest.mark.parametrize("B,S,P,nh,drop_p", [(3, 40, 256, 8, 0.0), (4, 499, 768, 8, 0.1)])
def test_xattn_two_query_sets(ops, B, S, P, nh, drop_p):
    """Positive + corrupted transcript queries over one audio K/V in one launch (engine's
    text->audio call, ref:training/trainer_unfreeze.py:525-542): each set equals its own
    single-query attention with its own dropout seed; dK/dV are the sum over both sets."""
    torch.manual_seed(S)
    q = torch.randn(2 * B, P, device=DEV)
    kv = torch.randn(B * S, 2 * P, device=DEV).bfloat16()
    k, v = kv[:, :P], kv[:, P:]
    mask = torch.ones(B * S, dtype=torch.int32, device=DEV)
    mask[S - 9:S] = 0
    mask[S:2 * S] = 0   # an all-masked sample: uniform probabilities, no score gradient (masked_fill)
    probs = torch.empty(2 * B * nh * S, device=DEV)
    out = torch.empty(2 * B, P, device=DEV)
    seeds = (1234, 777)
    ops.xattn_fwd(q, k, v, mask, B, S, nh, probs, out, seeds, drop_p=drop_p)
    d = P // nh
    qr = q.clone().requires_grad_()
    kr = k.float().clone().requires_grad_()
    vr = v.float().clone().requires_grad_()
    kh = kr.view(B, S, nh, d).transpose(1, 2)
    vh = vr.view(B, S, nh, d).transpose(1, 2)
    refs = []
    for qi in range(2):
        qh = qr[qi * B:(qi + 1) * B].view(B, 1, nh, d).transpose(1, 2)
        a = (qh @ kh.transpose(-2, -1)) * d ** -0.5
        a = a.masked_fill(mask.view(B, 1, 1, S) == 0, -1e9).softmax(-1)
        if drop_p > 0:
            idx = np.arange(B * nh * S).astype(np.uint64)
            a = a * torch.from_numpy(drop_scale(seeds[qi], idx, drop_p)).to(DEV).view(B, nh, 1, S)
        refs.append((a @ vh).transpose(1, 2).reshape(B, P))
    ref = torch.cat(refs)
    assert rel_err(out, ref) < 1e-5
    do = torch.randn(2 * B, P, device=DEV)
    ref.backward(do)
    dq = torch.empty(2 * B, P, device=DEV)
    dkv = torch.zeros(B * S, 2 * P, device=DEV)
    ops.xattn_bwd(q, k, v, probs, do, B, S, nh, dq, dkv[:, :P], dkv[:, P:], seeds, drop_p=drop_p, mask=mask)
    assert rel_err(dq, qr.grad) < 1e-5
    assert rel_err(dkv[:, :P], kr.grad) < 1e-5
    assert rel_err(dkv[:, P:], vr.grad) < 1e-5
    # bf16 variant (engine path): dK/dV written in bf16, their fp32 column sums (the fused
    # key/value bias gradient) added into a [2P] vector; nq=1 through xattn1_bwd the same way
    dq2 = torch.empty_like(dq)
    dkvb = torch.full((B * S, 2 * P), 7.0, device=DEV).bfloat16()   # written, not accumulated
    cs = torch.full((2 * P,), 0.25, device=DEV)
    ops.xattn_bwd(q, k, v, probs, do, B, S, nh, dq2, dkvb[:, :P], dkvb[:, P:], seeds, drop_p=drop_p, colsum=cs,
                  mask=mask)
    assert torch.equal(dq2, dq)
    assert torch.equal(dkvb, dkv.bfloat16())
    assert rel_err(cs - 0.25, dkv.sum(0)) < 1e-5
    dq1 = torch.empty(B, P, device=DEV)
    dkv1 = torch.zeros(B * S, 2 * P, device=DEV)
    ops.xattn1_bwd(q[:B], k, v, probs[:B * nh * S], do[:B], B, S, nh, dq1, dkv1[:, :P], dkv1[:, P:], drop_p=drop_p,
                   seed=seeds[0], mask=mask)
    dkv1b = torch.empty(B * S, 2 * P, device=DEV).bfloat16()
    cs1 = torch.zeros(2 * P, device=DEV)
    ops.xattn1_bwd(q[:B], k, v, probs[:B * nh * S], do[:B], B, S, nh, dq1, dkv1b[:, :P], dkv1b[:, P:],
                   drop_p=drop_p, seed=seeds[0], colsum=cs1, mask=mask)
    assert torch.equal(dkv1b, dkv1.bfloat16())
    assert rel_err(cs1, dkv1.sum(0)) < 1e-5


@pytest.mark.parametrize("B,L,T,P,drop_p", [(2, 12, 49, 128, 0.0), (3, 64, 499, 768, 0.0), (2, 20, 130, 256, 0.1)])
def test_align_attn(ops, B, L, T, P, drop_p):
    """WordLevelAlignmentModule's nn.MultiheadAttention core (4 heads, key padding mask,
    probability dropout) fwd + bwd vs torch fp32 (ref:training/trainer_unfreeze.py:285-292)."""
    torch.manual_seed(L + T)
    nh = 4
    q = torch.randn(B * L, P, device=DEV).bfloat16()
    kv = torch.randn(B * T, 2 * P, device=DEV).bfloat16()
    mask = torch.ones(B * T, dtype=torch.int32, device=DEV)
    mask[T - T // 5:T] = 0  # first clip padded
    probs = torch.empty(B * nh * L * T, device=DEV)
    out = torch.empty(B * L, P, device=DEV, dtype=torch.bfloat16)
    seed = 7
    ops.align_attn_fwd(q, kv, mask, B, L, T, nh, probs, out, drop_p=drop_p, seed=seed)
    d = P // nh
    qr = q.float().clone().requires_grad_()
    kvr = kv.float().clone().requires_grad_()
    qh = qr.view(B, L, nh, d).transpose(1, 2)
    kh = kvr[:, :P].reshape(B, T, nh, d).transpose(1, 2)
    vh = kvr[:, P:].reshape(B, T, nh, d).transpose(1, 2)
    s = (qh @ kh.transpose(-2, -1)) / math.sqrt(d)
    s = s.masked_fill(mask.view(B, 1, 1, T) == 0, float("-inf"))
    pr = s.softmax(-1)
    assert rel_err(probs.view(B, nh, L, T), pr) < 1e-5
    if drop_p > 0:
        idx = np.arange(B * nh * L * T).astype(np.uint64)
        pr = pr * torch.from_numpy(drop_scale(seed, idx, drop_p)).to(DEV).view(B, nh, L, T)
    ref = (pr @ vh).transpose(1, 2).reshape(B * L, P)
    assert rel_err(out, ref) < 5e-3  # bf16 output
    do = torch.randn(B * L, P, device=DEV).bfloat16()
    ref.backward(do.float())
    dq = torch.empty(B * L, P, device=DEV, dtype=torch.bfloat16)
    dkv = torch.empty(B * T, 2 * P, device=DEV)
    dsbuf = torch.empty(B * nh * L * T, device=DEV)
    ops.align_attn_bwd(q, kv, probs, do, B, L, T, nh, dsbuf, dq, dkv, drop_p=drop_p, seed=seed)
    assert rel_err(dq, qr.grad) < 5e-3
    assert rel_err(dkv, kvr.grad) < 1e-5


def test_rank1_bwd(ops):
    """Backward of Linear(K -> 1) after ReLU/tanh: dz = a ⊗ w ⊙ act'(z), dw = aᵀz, db = Σa."""
    from speech_transcript_embeddings_amd import _lib
    torch.manual_seed(8)
    M, K = 300, 384
    a = torch.randn(M, device=DEV)
    w = torch.randn(K, device=DEV)
    z = torch.randn(M, K, device=DEV).relu().bfloat16()
    out = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    dw = torch.zeros(K, device=DEV)
    db = torch.zeros(1, device=DEV)
    ops.rank1_bwd(a, w, z, _lib.ACT_RELU_BWD, out, dw, db)
    zf = z.float()
    assert rel_err(out, a[:, None] * w[None] * (zf > 0)) < 5e-3
    assert rel_err(dw, a @ zf) < 1e-5
    assert abs(db.item() - a.sum().item()) < 1e-3
    zt = torch.randn(M, K, device=DEV).tanh().bfloat16()
    ops.rank1_bwd(a, w, zt, _lib.ACT_TANH_BWD_OUT, out)
    assert rel_err(out, a[:, None] * w[None] * (1 - zt.float() ** 2)) < 5e-3


def test_loss_chain(ops):
    """normalize -> fp32-MFMA similarity -> AlignmentAwareInfoNCE, fwd + bwd vs torch."""
    torch.manual_seed(5)
    B, P, L = 20, 96, 9
    xa, xp, xn = (torch.randn(B, P, device=DEV) for _ in range(3))
    align = torch.randn(B, L, device=DEV)
    ya, yp, yn = (torch.empty(B, P, device=DEV) for _ in range(3))
    na, np_, nn_ = (torch.empty(B, device=DEV) for _ in range(3))
    for x, y, n in ((xa, ya, na), (xp, yp, np_), (xn, yn, nn_)):
        ops.l2norm_fwd(x, y, n)
    S = torch.empty(B, 2 * B, device=DEV)
    ops.similarity(ya, torch.cat([yp, yn]), S)
    sp, sn, loss = torch.empty(B, device=DEV), torch.empty(B, device=DEV), torch.empty(1, device=DEV)
    ops.pair_loss_fwd(S, B, align, B, L, 0.1, 0.5, 0.35, sp, sn, loss)
    xr = [t.clone().requires_grad_() for t in (xa, xp, xn, align)]
    a_, p_, n_ = (F.normalize(t, p=2, dim=1) for t in xr[:3])
    Sref = a_ @ torch.cat([p_, n_]).t()
    assert rel_err(S, Sref) < 1e-6
    spr, snr = (a_ * p_).sum(1), (a_ * n_).sum(1)
    logits = torch.stack([spr, snr], 1) / 0.1
    per = F.cross_entropy(logits, torch.zeros(B, dtype=torch.long, device=DEV), reduction="none")
    per = per * (1.0 - torch.sigmoid(xr[3].mean(1)) * 0.5)
    lref = per.mean() + 0.35 * F.relu(snr).mean()
    assert abs(loss.item() - lref.item()) < 1e-5 * max(1, abs(lref.item()))
    lref.backward()
    dsp, dsn = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    dalign = torch.empty(B, L, device=DEV)
    ops.pair_loss_bwd(sp, sn, align, B, L, 0.1, 0.5, 0.35, None, dsp, dsn, dalign)
    assert rel_err(dalign, xr[3].grad) < 1e-5
    dya, dyp, dyn = (torch.empty(B, P, device=DEV) for _ in range(3))
    ops.pair_sim_bwd(ya, yp, yn, dsp, dsn, dya, dyp, dyn)
    for y, n, dy, ref in ((ya, na, dya, xr[0]), (yp, np_, dyp, xr[1]), (yn, nn_, dyn, xr[2])):
        dx = torch.empty(B, P, device=DEV)
        ops.l2norm_bwd(y, n, dy, dx)
        assert rel_err(dx, ref.grad) < 1e-5


def test_text_embedding(ops):
    torch.manual_seed(6)
    B, L, D, V, pad = 3, 17, 128, 500, 1
    ids = torch.randint(5, V, (B, L), device=DEV)
    ids[1, 12:] = pad
    word = torch.randn(V, D, device=DEV)
    pos = torch.randn(514, D, device=DEV)
    typ = torch.randn(1, D, device=DEV)
    out = torch.empty(B * L, D, device=DEV)
    pid = torch.empty(B * L, dtype=torch.int32, device=DEV)
    ops.text_embed_fwd(ids, pad, word, pos, typ, out, pid)
    nz = (ids != pad).int()
    pref = (torch.cumsum(nz, 1) * nz).long() + pad
    assert torch.equal(pid.view(B, L).long(), pref)
    wr, pr, tr = (t.clone().requires_grad_() for t in (word, pos, typ))
    ref = F.embedding(ids, wr, padding_idx=pad) + tr[0] + F.embedding(pref, pr, padding_idx=pad)
    assert rel_err(out, ref.view(B * L, D)) < 1e-6
    do = torch.randn(B * L, D, device=DEV)
    ref.backward(do.view(B, L, D))
    dw, dp_, dt = torch.zeros_like(word), torch.zeros_like(pos), torch.zeros_like(typ)
    ops.text_embed_bwd(ids, pid, do, pad, dw, dp_, dt)
    assert rel_err(dw, wr.grad) < 1e-6
    assert rel_err(dp_, pr.grad) < 1e-6
    assert rel_err(dt, tr.grad) < 1e-6


def test_adamw_clip(ops):
    torch.manual_seed(8)
    n = 100003
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV) * 0.01
    m = torch.randn(n, device=DEV) * 1e-3
    v = torch.rand(n, device=DEV) * 1e-5
    acc = torch.zeros(1, device=DEV, dtype=torch.float64)
    ops.sumsq(g, acc)
    assert abs(acc.item() - (g.double() ** 2).sum().item()) < 1e-6 * acc.item()
    pr = p.clone().requires_grad_()
    opt = torch.optim.AdamW([pr], lr=1e-3, weight_decay=0.01)
    opt.state[pr] = {"step": torch.tensor(4.0), "exp_avg": m.clone(), "exp_avg_sq": v.clone()}
    total = acc.sqrt().item()
    pr.grad = g * min(1.0, 0.05 / (total + 1e-6))
    opt.step()
    pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ops.adamw(p, g, m, v, pb, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.01, step=5, sumsq_acc=acc,
              max_norm=0.05)
    assert rel_err(p, pr.detach()) < 1e-6
    assert torch.equal(pb, p.bfloat16())


def test_adamw_split_invariant(ops):
    """The update of an element does not depend on how the flat buffer is cut into launches (bulk
    two-group loop, one-group loop, scalar tail all round alike): TrainStep(overlap_optimizer=True)
    runs AdamW per parameter block and must match the one-launch-per-group update bit for bit."""
    torch.manual_seed(9)
    n = 3_000_011
    p0 = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV) * 0.01
    m0 = torch.randn(n, device=DEV) * 1e-3
    v0 = torch.rand(n, device=DEV) * 1e-5
    acc = torch.zeros(1, device=DEV, dtype=torch.float64)
    ops.sumsq(g, acc)
    kw = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.01, step=3, sumsq_acc=acc, max_norm=1.0)
    outs = []
    for cuts in ([0, n], [0, 4, 1_048_580, 1_048_600, 2_999_996, n], [0, 123_456, 2_000_000, n]):
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
        for a, b in zip(cuts, cuts[1:]):
            ops.adamw(p[a:b], g[a:b], m[a:b], v[a:b], pb[a:b], **kw)
        outs.append((p, m, v, pb))
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)
