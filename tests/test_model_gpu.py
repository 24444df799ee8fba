"""End-to-end parity of the HIP model (through libste.so) against the CPU oracle and the
reference's golden fixtures, at the golden mini dimensions (head_dim 64 like the real
encoders).  bf16 MFMA path: north_star's bf16 bound, 1e-2 relative on embeddings, loss and
per-tensor gradient norms; elementwise gradients checked against the oracle with the bounds
written in each test."""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN
from kref import bf16_exact
from oracle import det_init, ref_model as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def mini_model(meta, exact=False, **kw):
    """exact: bf16-representable weights (kref.bf16_exact), for elementwise parity vs the oracle."""
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.modules import AudioConfig, TextConfig
    m = meta["mini"]
    au, tx = m["audio"], m["text"]
    acfg = AudioConfig(hidden_size=au["hidden_size"], num_hidden_layers=au["num_hidden_layers"],
                       num_attention_heads=au["num_attention_heads"], intermediate_size=au["intermediate_size"],
                       mask_time_prob=0.0, layerdrop=0.0)
    tcfg = TextConfig(vocab_size=tx["vocab_size"], hidden_size=tx["hidden_size"],
                      num_hidden_layers=tx["num_hidden_layers"], num_attention_heads=tx["num_attention_heads"],
                      intermediate_size=tx["intermediate_size"])
    model = EnhancedAudioTextModel(text_model_name=tcfg, audio_model_name=acfg, projection_dim=m["projection_dim"],
                                   text_embedding_dim=tx["hidden_size"], audio_embedding_dim=au["hidden_size"],
                                   use_word_alignment=meta["use_word_alignment"], text_layers_to_unfreeze=m["unfreeze"],
                                   audio_layers_to_unfreeze=m["unfreeze"],
                                   use_attentive_pooling=meta.get("use_attentive_pooling", True), **kw)
    sd = model.state_dict()
    vals = det_init.state_dict_values([(n, t.shape) for n, t in sd.items()])
    model.load_state_dict({n: torch.from_numpy(bf16_exact(v) if exact else v) for n, v in vals.items()})
    return model


def oracle_params(meta, exact=False):
    cfg = R.mini_cfg(meta)
    vals = det_init.state_dict_values(R.param_shapes(cfg, spec_augment=False))
    return {n: torch.from_numpy(bf16_exact(v) if exact else v).requires_grad_(n in set(meta["trainable"]))
            for n, v in vals.items()}


def load(tag):
    meta = json.loads((GOLDEN / f"model_golden_{tag}.json").read_text())
    return meta, np.load(GOLDEN / f"model_golden_{tag}.npz")


def batch_of(z, dev=DEV):
    keys = ["input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
            "attention_mask_audio"]
    return {k: torch.from_numpy(z[k]).to(dev) for k in keys}


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def test_module_tree_matches_reference():
    meta, _ = load("noalign")
    model = mini_model(meta)
    assert list(model.state_dict().keys()) == meta["names"]
    tr = [n for n, p in model.named_parameters() if p.requires_grad]
    assert sorted(tr) == sorted(meta["trainable"])


def _grad_errors(model, meta, batch_cpu):
    cfg = R.mini_cfg(meta)
    vals = det_init.state_dict_values(R.param_shapes(cfg, spec_augment=False))
    p = {n: torch.from_numpy(v).requires_grad_(n in set(meta["trainable"])) for n, v in vals.items()}
    lo, *_ = R.step_loss(p, batch_cpu, cfg)
    lo.backward()
    params = dict(model.named_parameters())
    out = []
    for n in meta["with_grad"]:
        g_ref = p[n].grad
        if g_ref.norm() < 1e-6:
            continue
        out.append((rel(params[n].grad, g_ref), n))
    return sorted(out, reverse=True), lo.item()


@pytest.mark.parametrize("tag", ["noalign", "align", "nopool", "masked"])
def test_backward_random_cotangents(tag):
    """Backward of the whole model for random output cotangents vs the oracle's autograd.

    The real loss's cotangent on the audio embedding is ds*(t_neg - t_pos): a difference of
    two nearly identical vectors (the corrupted transcript, and random-init encoders make all
    embeddings close), which amplifies bf16 forward rounding.  Random cotangents exercise the
    same backward schedule without that cancellation, so this is the elementwise check of the
    backward at the bf16 rounding level; the loss-derived cotangents are checked exactly in
    test_kernels_gpu.py::test_loss_chain (fp32).  Both sides run on the same bf16-exact weights
    (kref.bf16_exact), so the comparison measures the kernels' arithmetic: every per-tensor error
    within north_star's 1e-2 bf16 bound."""
    meta, z = load(tag)
    model = mini_model(meta, exact=True)
    model.eval()
    from speech_transcript_embeddings_amd import align as A
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    cap = {}
    fwd = A.align_forward

    def capture(*a, **k):  # keep the HIP path's confidence-MLP hidden units (its ReLU gate)
        r = fwd(*a, **k)
        cap["c1"] = a[-1]["align"]["c1"].float().cpu()
        return r

    A.align_forward = capture
    try:
        bc = {k: torch.from_numpy(z[k]) for k in ["input_ids_pos", "attention_mask_pos", "input_ids_neg",
                                                   "attention_mask_neg", "input_values", "attention_mask_audio"]}
        batch = {k: v.to(DEV) for k, v in bc.items()}
        outs = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
    finally:
        A.align_forward = fwd
    g = torch.Generator().manual_seed(11)
    cots = [torch.randn(o.shape, generator=g) for o in outs]
    if model.last_alignment_scores is not None:
        outs = tuple(outs) + (model.last_alignment_scores,)
        cots.append(torch.randn(model.last_alignment_scores.shape, generator=g))
    torch.autograd.backward(outs, [c.to(DEV) for c in cots])
    cfg = R.mini_cfg(meta)
    p = oracle_params(meta, exact=True)
    tpn, tnn, an, align = R.compute_pos_neg_embeddings(p, bc, cfg)
    flips = 0
    if align is not None:
        assert rel(model.last_alignment_scores, align) < 2e-2
        # The alignment confidence MLP's ReLU is a discrete gate over b*L x P/2 = 24 x 64 hidden
        # units; the few pre-activations within bf16 rounding of zero flip it, and each flip moves
        # a 24-row gradient sum by O(1/sqrt(24)) (7-9 % on the head's grads).  To check the backward
        # schedule at the rounding level, re-run the oracle with the HIP path's gate.
        gate = (cap["c1"] > 0).float()

        class _Gated:
            def __getattr__(self, name):
                return getattr(F, name)

            @staticmethod
            def relu(x):
                nonlocal flips
                flips = int(((x.detach().reshape(gate.shape) > 0).float() != gate).sum())
                return x * gate.view(x.shape)

        R_F, R.F = R.F, _Gated()
        try:
            tpn, tnn, an, align = R.compute_pos_neg_embeddings(p, bc, cfg)
        finally:
            R.F = R_F
        assert flips < 0.01 * gate.numel(), flips
    ro = [tpn, tnn, an] + ([align] if align is not None else [])
    torch.autograd.backward(ro, cots)
    params = dict(model.named_parameters())
    errs = []
    for n in meta["with_grad"]:
        if p[n].grad.norm() < 1e-6:
            continue
        errs.append((rel(params[n].grad, p[n].grad), n))
    errs.sort(reverse=True)
    print(f"[{tag}] random-cotangent grad errors, bf16-exact weights (gate flips {flips}), worst:", errs[:6],
          "median:", errs[len(errs) // 2])
    # measured worst 0.77 / 1.12 / 0.65 / 0.87 % (noalign / align / nopool / masked).  With the
    # alignment head, its text_projection bias (the end of a chain of ten bf16 rounding points,
    # summed over L x heads of a gated MLP's rows) is checked against the bf16 floor of this
    # instance: the head re-run on the CPU with bf16 rounding at align.py's rounding points and the
    # HIP path's gate (tests/precision_probe_align.py, same weights, inputs and cotangents), vs
    # the same head in fp32 (measured emulated floor 1.06 %); every other tensor within 1e-2
    bound_head = 1e-2
    if tag == "align":
        import precision_probe_align as PA
        gs = {"gate": gate}
        ref_e = PA.run(meta, z, {f: False for f in PA.FLAGS}, gs)
        hip_e = PA.run(meta, z, {f: True for f in PA.FLAGS}, gs)
        floor = sorted(((rel(hip_e[n], ref_e[n]), n) for n in ref_e if ref_e[n].norm() > 1e-6), reverse=True)
        bound_head = max(1e-2, floor[0][0] + 1e-3)
        print(f"[{tag}] alignment head same-instance bf16 floor (emulated): worst {floor[:3]}; bound {bound_head:.4f}")
    for e, n in errs:
        assert e < (bound_head if n.startswith("word_level_alignment.") else 1e-2), (n, e)
    assert errs[len(errs) // 2][0] < 5e-3


@pytest.mark.parametrize("tag,precise_bwd", [("noalign", False), ("align", False), ("nopool", False), ("masked", False),
                                             ("nopool", True), ("masked", True)])
def test_forward_backward_matches_golden_and_oracle(tag, precise_bwd):
    """The drop-in autograd path (compute_pos_neg_embeddings -> (aud*txt).sum(1) -> loss_fn ->
    loss.backward(), ref :1068-1094) against the reference's golden outputs and the oracle.

    Forward: embeddings, s_pos, loss and alignment scores within 1e-2 of the reference's golden
    values (north_star's bf16 bound; measured <= 0.34 %).

    Backward, loss-derived: every gradient's norm within 1e-2 of the golden norm (measured worst
    0.30 / 0.40 / 0.29 % for noalign / align / nopool), and elementwise against the oracle's fp32
    autograd on the same batch and the same bf16-exact weights: per-tensor relative L2 error
    median < 1e-2 and worst < 2e-2, or the instance's emulated bf16 floor + 0.2 points where that is
    higher (measured median 0.3-0.7 %, worst 1.2-2.0 %; precise text backward: text tensors 1e-2),
    and >= 99 % of all gradient entries
    with the reference's sign (measured 99.75-99.8 %).  These gradients are sums of nearly
    cancelling positive- and corrupted-transcript terms (80 % shared tokens, random-init
    encoders), which amplify forward rounding; the heads run in fp32 and the text encoder's
    forward to ~fp32 accuracy for that reason (profiles/r3_parity.txt)."""
    meta, z = load(tag)
    model = mini_model(meta)
    model.eval()
    model.engine.precise_text_bwd = precise_bwd
    from speech_transcript_embeddings_amd.model import AlignmentAwareInfoNCE, EnhancedAudioTextModel
    batch = batch_of(z)
    tpn, tnn, an = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
    align = model.last_alignment_scores
    s_pos = (an * tpn).sum(1)
    s_neg = (an * tnn).sum(1)
    loss = AlignmentAwareInfoNCE(0.1, 0.5)(s_pos, s_neg, alignment_scores=align)
    loss.backward()
    torch.cuda.synchronize()
    errs = {"txt_pos": rel(tpn, z["txt_pos"]), "txt_neg": rel(tnn, z["txt_neg"]), "aud": rel(an, z["aud"]),
            "s_pos": rel(s_pos, z["s_pos"]), "loss": rel(loss.item(), float(z["loss"]))}
    if "align" in z.files:
        errs["align"] = rel(align, z["align"])
    print("forward rel errors vs reference golden:", errs)
    for k, v in errs.items():
        assert v < 1e-2, (k, v)
    params = dict(model.named_parameters())
    for n, prm in params.items():
        if n not in set(meta["with_grad"]):
            assert prm.grad is None, n
    worst = []
    for n in meta["with_grad"]:
        gn = float(z[f"gnorm::{n}"])
        g_gpu = params[n].grad
        assert g_gpu is not None, n
        if gn < 1e-6:  # analytically ~0 (softmax shift-invariant biases): absolute check
            # only rounding noise (bf16 dK summed over rows); Adam maps such noise to ±lr
            # steps in the reference as well (tests/test_oracle_golden.py::test_optimizer...)
            assert g_gpu.abs().max().item() < 2e-3, n
            continue
        worst.append((abs(g_gpu.double().norm().item() - gn) / gn, n))
    worst.sort(reverse=True)
    print(f"[{tag}] gradient-norm errors vs golden: worst {worst[:4]}, median {worst[len(worst) // 2][0]:.2e}")
    assert worst[0][0] < 1e-2, worst[:4]
    # elementwise against the oracle's fp32 autograd of the same loss (pinned to the golden), both
    # on the same bf16-exact weights (kref.bf16_exact: the kernels' arithmetic, not the weights'
    # bf16 quantisation, which the golden-norm check above already covers)
    cfg = R.mini_cfg(meta)
    p = oracle_params(meta, exact=True)
    bc = {k: v.cpu() for k, v in batch.items()}
    lo, *_ = R.step_loss(p, bc, cfg)
    lo.backward()
    mx = mini_model(meta, exact=True)
    mx.eval()
    mx.engine.precise_text_bwd = precise_bwd
    tpx, tnx, anx = EnhancedAudioTextModel.compute_pos_neg_embeddings(mx, batch)
    AlignmentAwareInfoNCE(0.1, 0.5)((anx * tpx).sum(1), (anx * tnx).sum(1),
                                    alignment_scores=mx.last_alignment_scores).backward()
    torch.cuda.synchronize()
    px = dict(mx.named_parameters())
    errs, agree, total = [], 0, 0
    for n in meta["with_grad"]:
        g_ref = p[n].grad.double().reshape(-1)
        if g_ref.norm() < 1e-6:
            continue
        g_hip = px[n].grad.detach().double().cpu().reshape(-1)
        errs.append((rel(g_hip, g_ref), n))
        agree += int((torch.sign(g_hip) == torch.sign(g_ref)).sum())
        total += g_ref.numel()
    errs.sort(reverse=True)
    print(f"[{tag}] elementwise vs oracle, bf16-exact weights: worst {errs[:3]}, median {errs[len(errs) // 2][0]:.2e}, "
          f"sign agreement {agree / total:.5f}")
    # measured worst 1.18 / 1.17 / 2.01 / 1.36 % (noalign / align / nopool / masked), all on the
    # trainable text layer's attention and the token-type row: the loss gradient there is the
    # difference of the clean and corrupted transcripts' nearly equal backward passes (80 % shared
    # tokens), and the text backward's bf16 dY operands carry that cancellation.  The
    # bound is 2e-2, or — where that is the bf16 floor itself — the floor of this instance + 0.2
    # points: the oracle's step re-run on the CPU with bf16 rounding at the HIP path's rounding
    # points (tests/precision_probe_text.py, set "all": the text backward's dY / dO / P-dS / dW
    # operands and the audio encoder's bf16 forward storage) against fp32.  nopool's emulated floor
    # is 1.90 % on the text value bias (the GPU reads 1.68-2.03 % there across trees that leave the
    # text path unchanged: the cancellation amplifies rounding-order differences); the other golden
    # cases' floors are 0.70-0.94 %, below the GPU's 1.17-1.36 %, so 2e-2 holds them
    bound = 2e-2
    if not precise_bwd:
        import precision_probe_text as PT
        ref_t = PT.run(meta, z, {f: False for f in PT.FLAGS})
        hip_t = PT.run(meta, z, {f: True for f in PT.FLAGS})
        floor = sorted(((rel(hip_t[n], ref_t[n]), n) for n in ref_t if ref_t[n].norm() > 1e-6), reverse=True)
        bound = max(2e-2, floor[0][0] + 2e-3)
        print(f"[{tag}] loss-derived same-instance bf16 floor (emulated): worst {floor[:3]}; bound {bound:.4f}")
    assert errs[len(errs) // 2][0] < 1e-2 and errs[0][0] < bound, errs[:3]
    assert agree >= 0.99 * total, agree / total
    if precise_bwd:
        # the precise text backward (fp32 attention backward, split dY / dW operands): every text
        # gradient within north_star's 1e-2 bf16 bound (measured 0.20 / 0.37 %, masked / nopool; with the bf16 text
        # backward 1.1-2.0 %, tests/precision_probe_text.py attributes it to the dY / dO rounding)
        text = [(e, n) for e, n in errs if n.startswith("text_encoder.")]
        print(f"[{tag}] precise text backward, text tensors worst {text[:3]}")
        assert text[0][0] < 1e-2, text[:3]


def test_fp8_gemm_matches_oracle():
    """fp8_gemm=True (BASELINE config 5): the Conformer forward GEMMs run MX-fp8 (e4m3, 32-k
    block scales); gradients stay bf16 (straight-through).  Parity bound for this precision
    (north_star states fp32/bf16 only; stated here): embeddings and loss within 5e-2 relative of
    the fp32 oracle, per-tensor gradient norms within 10 %."""
    meta, z = load("noalign")
    from speech_transcript_embeddings_amd.model import AlignmentAwareInfoNCE, EnhancedAudioTextModel
    model = mini_model(meta, fp8_gemm=True)
    model.eval()
    batch = batch_of(z)
    tpn, tnn, an = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
    s_pos, s_neg = (an * tpn).sum(1), (an * tnn).sum(1)
    loss = AlignmentAwareInfoNCE(0.1, 0.5)(s_pos, s_neg)
    loss.backward()
    torch.cuda.synchronize()
    errs = {"txt_pos": rel(tpn, z["txt_pos"]), "aud": rel(an, z["aud"]), "s_pos": rel(s_pos, z["s_pos"]),
            "loss": rel(loss.item(), float(z["loss"]))}
    print("fp8 forward rel errors vs reference golden:", errs)
    for k, v in errs.items():
        assert v < 5e-2, (k, v)
    # the MX-fp8 path really ran: the cached quantised weights exist for every Conformer Linear
    n_q = len(model.store._wq)  # FFN1 in/out, QKV, O, pw1, pw2, FFN2 in/out per layer
    assert n_q == 8 * meta["mini"]["audio"]["num_hidden_layers"], n_q
    params = dict(model.named_parameters())
    worst = []
    for n in meta["with_grad"]:
        gn = float(z[f"gnorm::{n}"])
        if gn < 1e-6:
            continue
        worst.append((abs(params[n].grad.double().norm().item() - gn) / gn, n))
    worst.sort(reverse=True)
    print("worst fp8 grad-norm errors:", worst[:5])
    assert worst[0][0] < 0.1, worst[0]


def test_gradient_accumulation_matches_full_batch():
    """TrainStep(accumulation_steps=N) (ref train_epoch :1064-1117): N micro-batches of b with
    loss/N summed into the gradient buffer equal one batch of N*b (the loss is a per-sample
    mean), the optimizer steps once per window, and flush() steps on a partial window with the
    reference's 1/N scaling (ref :1064-1066 is_last_batch).  Dropout off so both runs see the
    same function; no clipping (clip_grad_norm_ would rescale).  Power-of-two N scale every bf16
    cotangent exactly, so those runs agree to fp32 summation order; N = 3 rounds the scaled
    cotangents differently, and the loss gradient's ds·(t_neg − t_pos) cancellation amplifies
    that bf16 rounding, so it is checked at the gradient-norm level."""
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    meta, _ = load("noalign")

    def build():
        m = mini_model(meta, spec_augment=False)
        m.dropout = 0.0
        m.audio_cfg.conformer_conv_dropout = 0.0
        m.audio_cfg.layerdrop = 0.0
        m.text_cfg.hidden_dropout_prob = 0.0
        m.text_cfg.attention_probs_dropout_prob = 0.0
        return m

    data = synthetic_batch(4, 16000, 12, vocab=meta["mini"]["text"]["vocab_size"], seed=3)
    halves = [tuple(t[:2] for t in data), tuple(t[2:] for t in data)]

    def run(acc, seq, flush=False):
        m = build()
        st = TrainStep(m, lr=1e-3, warmup=1, total_steps=10, accumulation_steps=acc, max_norm=1e9)
        for k, i in enumerate(seq):
            st(*halves[i])
            assert st.opt.t == (k + 1) // acc
        if flush:
            assert st.flush() and not st.flush()
        assert st.opt.t == 1 and st._micro == 0
        torch.cuda.synchronize()
        return m.store.grad.clone()

    m1 = build()
    s1 = TrainStep(m1, lr=1e-3, warmup=1, total_steps=10, max_norm=1e9)
    s1(*data)
    torch.cuda.synchronize()
    g_full = m1.store.grad.clone()
    assert rel(run(2, [0, 1]), g_full) < 1e-5  # fp32 summation order (1.0e-6 measured)
    assert rel(run(4, [0, 1], flush=True), g_full * 0.5) < 1e-5
    g3 = run(3, [0, 1], flush=True)
    assert abs(g3.norm().item() / (g_full.norm().item() * 2.0 / 3.0) - 1.0) < 2e-2


@pytest.mark.parametrize("tag", ["noalign", "align"])
def test_train_step_matches_reference_optimizer_step(tag):
    """The benched fused step (TrainStep: fwd -> L2 norm -> B x 2B similarity -> pair loss ->
    backward -> clip_grad_norm_(1.0) folded into the two-group AdamW -> warmup schedule) against
    the REFERENCE's own optimizer tail on the golden mini batch (make_golden.py: the reference
    model's loss.backward(), clip_grad_norm_, torch AdamW with encoder lr/50 and heads lr, and
    get_linear_schedule_with_warmup at scheduler step 1; ref :1084-1117, :1487-1541).
    Eval numerics (every dropout 0, no SpecAugment, no layerdrop) so both sides run the same
    function.  Checked:
      * loss within 1e-2, clip_grad_norm_'s total norm within 1e-2 (measured 4e-5 / 4e-4);
      * both groups' learning rates exactly (lr/50 and lr at warmup factor 1/2);
      * the updated parameters at the golden's sampled entries.  AdamW's first step from zero
        moments moves each entry by lr·g/(|g| + eps) ≈ ±lr, so the new value depends only on
        the SIGN of its clipped gradient.  (a) Given the HIP gradient the fused clip + AdamW +
        schedule is exact (1e-6); (b) against the reference's updated values every entry differs
        by exactly lr·|u_hip - u_ref|, u = g/(|g| + eps) of each side's clipped gradient — only
        through the gradients — and the update directions (the gradient signs) agree on >= 99 %
        of the sampled entries (measured 99.6 %)."""
    from speech_transcript_embeddings_amd.train import TrainStep
    meta, z = load(tag)
    model = mini_model(meta, spec_augment=False)
    model.dropout = 0.0
    model.audio_cfg.conformer_conv_dropout = 0.0
    model.audio_cfg.layerdrop = 0.0
    model.text_cfg.hidden_dropout_prob = 0.0
    model.text_cfg.attention_probs_dropout_prob = 0.0
    params = dict(model.named_parameters())
    before = {n: params[n].detach().clone().reshape(-1) for n in meta["with_grad"]}
    step = TrainStep(model, lr=meta["lr"], warmup=meta["warmup"], total_steps=meta["total_steps"])
    step.sched.step_count = meta["sched_step"]   # the reference took the step at scheduler step 1
    loss = step.step_batch(batch_of(z))
    torch.cuda.synchronize()
    assert step.opt.t == 1 and step.sched.step_count == meta["sched_step"] + 1
    assert rel(loss.item(), float(z["loss"])) < 1e-2
    tn = step.opt.total_norm()
    print(f"[{tag}] loss {loss.item():.6f} vs {float(z['loss']):.6f}; clip total norm {tn:.6f} vs "
          f"{float(z['clip_total_norm']):.6f}")
    assert rel(tn, float(z["clip_total_norm"])) < 1e-2
    f = step.opt.last_factor
    lr_enc, lr_head = step.opt.groups[0]["lr"] * f, step.opt.groups[1]["lr"] * f
    assert abs(lr_enc - float(z["lr_enc"])) <= 1e-12 and abs(lr_head - float(z["lr_head"])) <= 1e-12
    coef = min(1.0, 1.0 / (tn + 1e-6))
    coef_ref = min(1.0, 1.0 / (float(z["clip_total_norm"]) + 1e-6))
    agree = total = 0
    for n in meta["with_grad"]:
        lr = lr_enc if ("text_encoder" in n or "audio_encoder" in n) else lr_head
        idx = det_init.sample_indices(n, before[n].numel())
        it = torch.from_numpy(idx).to(DEV)
        new = params[n].detach().reshape(-1)[it].double().cpu().numpy()
        p0 = before[n][it].double().cpu().numpy()
        g = model.store.g(n).reshape(-1)[it].double().cpu().numpy() * coef
        # (a) the fused clip + AdamW + schedule is exact given the HIP gradient (torch AdamW's
        #     first step from zero moments: decay, then lr·m̂/(sqrt(v̂) + eps) = lr·g/(|g| + eps))
        want = p0 * (1 - lr * 0.01) - lr * g / (np.abs(g) + 1e-8)
        assert np.abs(new - want).max() <= 1e-6, (n, np.abs(new - want).max())
        # (b) against the reference's updated values: the two updates differ exactly by
        #     lr·|u_hip - u_ref| with u = g/(|g| + eps) of each side's clipped gradient, i.e. only
        #     through the gradients themselves (identical where the signs agree and |g| >> eps)
        ref = z[f"pnew::{n}"].astype(np.float64)
        g_ref = z[f"gsamp::{n}"].astype(np.float64) * coef_ref
        u_h, u_r = g / (np.abs(g) + 1e-8), g_ref / (np.abs(g_ref) + 1e-8)
        assert np.all(np.abs(new - ref) <= lr * np.abs(u_h - u_r) + 2e-6), n
        # signs are compared where the reference gradient is not fp32 round-off: the key biases,
        # the pooling scorer's output bias and the key slice of in_proj_bias have analytically zero
        # gradients (softmax shift invariance) whose ±1e-10 values carry random signs — the oracle
        # and the reference agree on only 98 % of the sampled entries because of them
        gn = float(z[f"gnorm::{n}"])
        live = np.abs(g_ref) > 1e-6 * max(gn, 1e-30) if gn >= 1e-6 else np.zeros(g_ref.shape, bool)
        agree += int((np.sign(g) == np.sign(g_ref))[live].sum())
        total += int(live.sum())
    print(f"[{tag}] sampled entries whose gradient sign (hence update direction) agrees with the reference: "
          f"{agree}/{total} = {agree / total:.4f}")
    assert agree >= 0.99 * total
