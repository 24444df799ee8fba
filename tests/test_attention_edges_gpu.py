"""Attention at a single frame (T = 1), where the softmax is exactly 1 and the score gradients vanish
analytically (tests/test_kernels_gpu.py covers every other length)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from speech_transcript_embeddings_amd import ops as _ops
    return _ops


@pytest.mark.parametrize("rel", [False, True])
def test_attention_single_frame(ops, rel):
    """T = 1: one key, P = 1 exactly, so O = V, dV = dO, and dS = dP - delta = 0 analytically: dQ,
    dK (and dE) must vanish to the rounding of the two 64-term dot products (a relative error
    against the ~0 reference is meaningless here, so the bound is on |dS|·|K|)."""
    torch.manual_seed(11)
    B, T, H, D = 3, 1, 2, 64
    W = H * D
    qkv = (torch.randn(B * T, 3 * W, device=DEV) * 0.7).bfloat16()
    q, k, v = qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:]
    mask = torch.tensor([1, 0, 1], dtype=torch.int32, device=DEV)   # sample 1: its only key masked
    E = (torch.randn(73, D, device=DEV) * 0.5).bfloat16() if rel else None
    o = torch.empty(B * T, W, device=DEV, dtype=torch.bfloat16)
    olo = torch.empty_like(o)
    lse = torch.empty(B * H * T, device=DEV)
    ops.attention_fwd(q, k, v, B=B, T=T, H=H, o=o, lse=lse, key_mask=mask, rel_E=E, o_lo=olo)
    assert torch.equal(o, v) and torch.count_nonzero(olo) == 0
    do = torch.randn(B * T, W, device=DEV).bfloat16()
    dq, dk, dv = (torch.full((B * T, W), 5.0, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    dE = torch.zeros(73, D, device=DEV) if rel else None
    ops.attention_bwd(q, k, v, o, lse, do, dq, dk, dv, B=B, T=T, H=H, delta=torch.empty(B * H * T, device=DEV),
                      key_mask=mask, rel_E=E, dE=dE, gwork=torch.empty(B * H * T * 80, device=DEV) if rel else None,
                      o_lo=olo)
    assert torch.equal(dv, do)
    hv = lambda t: t.float().view(B * T, H, D)
    ds_bound = 1e-5 * hv(do).norm(dim=-1) * hv(v).norm(dim=-1)     # |dP - delta| per (row, head)
    for g, x in ((dq, k), (dk, q)):
        assert (hv(g).norm(dim=-1) <= ds_bound * hv(x).norm(dim=-1) * 0.125 + 1e-30).all()
    if rel:
        assert float(dE.norm()) <= float((ds_bound * hv(q).norm(dim=-1)).sum()) * 0.125
