"""The drop-in boundary on the GPU: the ste:: custom ops (torch_ops.py) against plain PyTorch
fp32 references, and the reference's own forward written against the public API.

* each op's forward and registered backward vs torch fp32 (bf16 MFMA operands: 1e-2-class
  tolerances; fp32 ops 1e-5), plus torch.library.opcheck (schema, fake tensor, autograd
  registration) for the differentiable ones;
* the reference's `_forward()` body (trainer_unfreeze.py:1068-1081) with the reference's
  compute_pos_neg_embeddings written out as in ref :508-563 — encode_text x2, encode_audio,
  apply_cross_modal_attention x2, F.normalize — on the differentiable sub-APIs, the loss on
  ste::pair_loss, then loss.backward(): embeddings and loss vs the reference's golden values and
  the fused single-node path, gradient norms vs the golden, and (random cotangents) every
  parameter gradient vs the fused path."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from kref import attention_ref
from test_model_gpu import batch_of, load, mini_model, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ste():
    import speech_transcript_embeddings_amd  # noqa: F401
    return torch.ops.ste


def test_linear_op(ste):
    torch.manual_seed(0)
    x = torch.randn(3, 50, 96, device=DEV, requires_grad=True)
    w = (torch.randn(80, 96, device=DEV) * 0.1).requires_grad_()
    b = torch.randn(80, device=DEV, requires_grad=True)
    y = ste.linear(x, w, b)
    xr, wr, br = (t.detach().bfloat16().float().requires_grad_() for t in (x, w, b))
    yr = xr @ wr.t() + b.detach()
    assert rel(y, yr) < 1e-5               # bf16 operands, fp32 accumulation
    dy = torch.randn_like(y)
    y.backward(dy)
    (yr * dy).sum().backward()
    assert rel(x.grad, dy.bfloat16().float() @ wr.detach()) < 1e-5
    assert rel(w.grad, dy.bfloat16().float().reshape(-1, 80).t() @ xr.detach().reshape(-1, 96)) < 1e-5
    assert rel(b.grad, dy.sum((0, 1))) < 1e-5
    torch.library.opcheck(ste.linear.default, (x.detach(), w.detach(), b.detach()),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


def test_layer_norm_op(ste):
    torch.manual_seed(1)
    x = torch.randn(6, 20, 1024, device=DEV, requires_grad=True)
    g = (1 + 0.1 * torch.randn(1024, device=DEV)).requires_grad_()
    b = (0.1 * torch.randn(1024, device=DEV)).requires_grad_()
    y, mean, rstd = ste.layer_norm(x, g, b, 1e-5)
    xr, gr, br = (t.detach().clone().requires_grad_() for t in (x, g, b))
    yr = F.layer_norm(xr, (1024,), gr, br, 1e-5)
    assert rel(y, yr) < 1e-5
    assert rel(mean, xr.detach().reshape(-1, 1024).mean(1)) < 1e-5
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    for a, r in ((x.grad, xr.grad), (g.grad, gr.grad), (b.grad, br.grad)):
        assert rel(a, r) < 1e-5
    torch.library.opcheck(ste.layer_norm.default, (x.detach(), g.detach(), b.detach(), 1e-5),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


@pytest.mark.parametrize("rel_bias", [True, False])
def test_attention_op(ste, rel_bias):
    torch.manual_seed(2)
    B, T, H = 2, 130, 2
    q, k, v = ((torch.randn(B, T, H * 64, device=DEV) * 0.5).bfloat16().requires_grad_() for _ in range(3))
    E = (torch.randn(73, 64, device=DEV) * 0.5).bfloat16().requires_grad_() if rel_bias else None
    mask = torch.ones(B, T, dtype=torch.int32, device=DEV)
    mask[1, 100:] = 0
    o, lse, o_lo = ste.attention(q, k, v, mask, E, 0.125, 64, 8)
    qf, kf, vf = (t.detach().float().view(B, T, H, 64).requires_grad_() for t in (q, k, v))
    Ef = E.detach().float().requires_grad_() if rel_bias else None
    ref = attention_ref(qf, kf, vf, mask, Ef)
    assert rel(o.float().view(B, T, H, 64), ref) < 1e-2
    assert rel(o.float() + o_lo.float(), ref.reshape(B, T, H * 64)) < 1e-4
    do = torch.randn(B, T, H * 64, device=DEV).bfloat16()
    o.backward(do)
    ref.backward(do.float().view(B, T, H, 64))
    for a, r in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        assert rel(a.float().view(B, T, H, 64), r) < 1e-2
    if rel_bias:
        assert rel(E.grad.float(), Ef.grad) < 1e-2


def test_pair_loss_op(ste):
    from oracle import ref_model as R
    torch.manual_seed(3)
    B, L = 8, 12
    sp = (torch.rand(B, device=DEV) * 2 - 1).requires_grad_()
    sn = (torch.rand(B, device=DEV) * 2 - 1).requires_grad_()
    al = torch.randn(B, L, device=DEV, requires_grad=True)
    for align in (None, al):
        loss = ste.pair_loss(sp, sn, align, 0.1, 0.5, 0.35)
        xs = [t.detach().double().cpu().requires_grad_() for t in (sp, sn)]
        ar = None if align is None else align.detach().double().cpu().requires_grad_()
        lr_ = R.alignment_aware_infonce(xs[0], xs[1], ar, temperature=0.1, alignment_weight=0.5, corrupt_gamma=0.35)
        assert abs(loss.item() - lr_.item()) < 1e-5
        gs = torch.autograd.grad(loss, [sp, sn] + ([al] if align is not None else []))
        grs = torch.autograd.grad(lr_, xs + ([ar] if ar is not None else []))
        for a, r in zip(gs, grs):
            assert rel(a, r) < 1e-5
    torch.library.opcheck(ste.pair_loss.default, (sp.detach(), sn.detach(), None, 0.1, 0.5, 0.35),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


def test_fbank_op_matches_reference_extractor(ste):
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, str(GOLDEN))
    from fbank_cases import long_case_wave
    z = np.load(GOLDEN / "fbank_golden_long.npz")
    w = torch.from_numpy(long_case_wave("10s")).to(DEV)[None]
    feats, mask = ste.fbank(w, torch.tensor([w.shape[1]], dtype=torch.int32, device=DEV), 499, 1.0, 1)
    np.testing.assert_allclose(feats[0].cpu().numpy(), z["10s_feats"], atol=5e-4, rtol=0)
    np.testing.assert_array_equal(mask[0].cpu().numpy(), z["10s_mask"])


def test_adamw_op(ste):
    from oracle import ref_model as R
    torch.manual_seed(4)
    n = 10000
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.randn(n, device=DEV) * 0.1
    v = torch.rand(n, device=DEV) * 0.01
    pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    sumsq = torch.tensor([(g.double() ** 2).sum().item()], device=DEV, dtype=torch.float64)
    p0, m0, v0 = p.clone(), m.clone(), v.clone()
    ste.adamw_(p, g, m, v, pb, 1e-3, 0.9, 0.999, 1e-8, 0.01, 5, sumsq, 1.0)
    coef = min(1.0, 1.0 / (math.sqrt(sumsq.item()) + 1e-6))
    pr, mr, vr = R.adamw_step(p0.cpu(), g.cpu() * coef, m0.cpu(), v0.cpu(), lr=1e-3, step=5)
    assert rel(p, pr) < 1e-6 and rel(m, mr) < 1e-6 and rel(v, vr) < 1e-6
    assert torch.equal(pb, p.bfloat16())


def _reference_compute_pos_neg_embeddings(model, batch):
    """ref :508-563 (use_word_alignment=False), written against the public methods."""
    txt_pos_proj, txt_pos_hidden = model.encode_text(batch["input_ids_pos"], batch["attention_mask_pos"])
    txt_neg_proj, txt_neg_hidden = model.encode_text(batch["input_ids_neg"], batch["attention_mask_neg"])
    aud_proj, aud_hidden = model.encode_audio(batch["input_values"], batch["attention_mask_audio"])
    if model.use_cross_modal:
        txt_pos_fused, aud_fused = model.apply_cross_modal_attention(
            txt_pos_proj, txt_pos_hidden, batch["attention_mask_pos"], aud_proj, aud_hidden,
            batch["attention_mask_audio"])
        txt_neg_fused, _ = model.apply_cross_modal_attention(
            txt_neg_proj, txt_neg_hidden, batch["attention_mask_neg"], aud_proj, aud_hidden,
            batch["attention_mask_audio"])
    else:
        txt_pos_fused, txt_neg_fused, aud_fused = txt_pos_proj, txt_neg_proj, aud_proj
    return (F.normalize(txt_pos_fused, p=2, dim=1), F.normalize(txt_neg_fused, p=2, dim=1),
            F.normalize(aud_fused, p=2, dim=1))


@pytest.mark.parametrize("tag", ["noalign", "nopool"])
def test_reference_forward_body_through_public_api(tag):
    """Forward: the reference's body gives the reference's golden embeddings and loss (1e-2), and
    the fused path's values (1e-5: same kernels, same rounding).  Backward: loss.backward() fills
    every gradient, with per-tensor norms vs the golden within the fused path's bound
    (test_model_gpu.py::test_forward_backward_matches_golden_and_oracle; loss-derived gradients
    are pos/neg cancellations, and this composition rounds the pos and neg cross-modal K/V
    gradients to bf16 separately where the fused path sums them first); for random output
    cotangents (no cancellation) every gradient matches the fused path's within 2e-2."""
    from speech_transcript_embeddings_amd.model import AlignmentAwareInfoNCE, EnhancedAudioTextModel
    meta, z = load(tag)
    batch = batch_of(z)
    loss_fn = AlignmentAwareInfoNCE(temperature=0.1, alignment_weight=0.5)

    def _forward(model, compute):   # ref :1068-1081
        txt_pos_norm, txt_neg_norm, aud_norm = compute(model, batch)
        s_pos = (aud_norm * txt_pos_norm).sum(dim=1)
        s_neg = (aud_norm * txt_neg_norm).sum(dim=1)
        alignment_scores = getattr(model, "last_alignment_scores", None)
        loss = loss_fn(s_pos, s_neg, alignment_scores=alignment_scores)
        return loss, s_pos, s_neg, (txt_pos_norm, txt_neg_norm, aud_norm)

    m1 = mini_model(meta)
    m1.eval()
    loss1, sp1, sn1, emb1 = _forward(m1, _reference_compute_pos_neg_embeddings)
    loss1.backward()
    m2 = mini_model(meta)
    m2.eval()
    loss2, sp2, sn2, emb2 = _forward(m2, EnhancedAudioTextModel.compute_pos_neg_embeddings)
    torch.cuda.synchronize()
    for name, got in zip(["txt_pos", "txt_neg", "aud"], emb1):
        assert rel(got, z[name]) < 1e-2, name
    assert rel(loss1.item(), float(z["loss"])) < 1e-2
    for a, b in zip(emb1, emb2):
        assert rel(a, b) < 1e-5
    p1 = dict(m1.named_parameters())
    worst = []
    for n in meta["with_grad"]:
        assert p1[n].grad is not None, n
        gn = float(z[f"gnorm::{n}"])
        if gn < 1e-6:
            continue
        worst.append((abs(p1[n].grad.double().norm().item() - gn) / gn, n))
    worst.sort(reverse=True)
    print(f"[{tag}] public-API composition, gradient-norm errors vs golden: {worst[:3]}")
    assert worst[0][0] < 1e-2, worst[:3]
    # random cotangents on both paths
    g = torch.Generator(device=DEV).manual_seed(7)
    cots = [torch.randn(e.shape, device=DEV, generator=g) for e in emb1]
    m1.zero_grad()
    m2.zero_grad()
    e1 = _reference_compute_pos_neg_embeddings(m1, batch)
    torch.autograd.backward(e1, cots)
    e2 = EnhancedAudioTextModel.compute_pos_neg_embeddings(m2, batch)
    torch.autograd.backward(e2, cots)
    torch.cuda.synchronize()
    p2 = dict(m2.named_parameters())
    errs = []
    for n in meta["with_grad"]:
        if p2[n].grad.norm() < 1e-6 or n.endswith(("key.bias", "linear_k.bias")):
            continue  # softmax shift invariance: true gradient 0
        errs.append((rel(p1[n].grad, p2[n].grad), n))
    errs.sort(reverse=True)
    print(f"[{tag}] random cotangents, public-API composition vs fused path: worst {errs[:3]}")
    assert errs[0][0] < 2e-2, errs[:3]
