"""Full-size parity at every BASELINE config's shapes (w2v-bert-2.0 24 x 1024 Conformer,
XLM-R-base 12 x 768 text encoder): the HIP path against the oracle's CPU fp32 autograd on the
SAME weights (the GPU model's own random init, copied to the oracle), eval mode.
  c1  B=4, 2 s clips, 16-token transcripts, 3+3 unfrozen
  c2  B=2, 10 s clips, 64 tokens, 3+3 unfrozen          (c3 = c2 shapes per GPU)
  c4  B=2, 10 s, 64 tokens, 5+5 unfrozen + alignment head
  c5  B=1, 30 s clips (T = 1499), 64 tokens, every encoder layer trainable (freeze_encoders
      "none"), bf16 GEMMs and, separately, the MX-fp8 Conformer forward GEMMs (fp8_gemm=True)

Checked: the three normalised embeddings and alignment scores (bf16 bound of north_star:
1e-2 relative), and the gradient of every parameter that receives one, for random cotangents
on the outputs (the loss-derived cotangent is a near-cancelling pos/neg difference, see
test_model_gpu.py::test_forward_backward_matches_golden_and_oracle).  Gradients are compared
tensor-wise by relative L2 norm of the difference; with the alignment head the oracle re-runs
with the HIP path's ReLU gate.

Weights: every config runs on bf16-exact weights (kref.bf16_exact: the same values on both
sides, representable in the GEMMs' operand format), so the comparison measures the kernels'
arithmetic; c2_fp32w repeats c2 end to end with arbitrary fp32 master weights, whose bf16
rounding the GEMMs read.  The bf16 floor of the reference graph (tests/precision_probe.py,
profiles/r4_bf16_floor.txt, CPU, c2 shapes): the fp32 graph with only its weights rounded to
bf16 moves the worst tensor by 1.33 %, with only the forward activations stored bf16 at the
HIP path's rounding points by ~1.0 %, and the reference under bf16 autocast by 4.8 %; the HIP
path is at 0.93 % (bf16-exact weights) / 1.8 % (fp32 weights).

The gradients cross all 24 Conformer layers (feature_projection is trainable) on bf16 MFMA
operands.  Random-init encoders produce activations that are nearly identical across frames
(a large common component), so every softmax backward dS = P(dP - delta) is a small
difference of large terms: delta is formed from the ~fp32 attention output (ste_attn_args.o_lo,
the forward's PV product on P = hi + lo), which took the q/k projections of the deepest
trainable layer from 3.3 % to 1.7 %.  The audio attentive-pooling scorer runs on the encoder
output's [hi | lo] split image with fp32 tanh activations (r3: 2.3 % -> 1.75 %); what is left
there is the bf16 audio encoder's forward rounding of that common component (the scorer's
gradient Σ_l dz_l ⊗ h_l cancels across frames), the same limit as the deepest layers' q/k.

The floor of THIS instance (round 5).  How far a bf16 path can get from fp32 on these tensors
depends on the draw: the CPU probe's emulation of the HIP rounding points (tests/precision_probe.py,
bf16-exact weights, c1 shapes) puts the worst tensor anywhere in 0.89-1.37 % over seeds 0-5
(profiles/r5_parity.txt), so a floor measured on another draw says little about this one.  The
bf16-exact configs therefore emulate the floor on the test's own weights, clips and cotangents:
the audio encoder + pooling run again on the CPU with bf16 rounding at the HIP path's rounding
points (precision_probe.Probe: forward activations, backward dY / dX operands, attention dS and
P, the FFN pre-activation the swish backward reads) and in fp32, driven by the cotangents the
fp32 oracle's backward delivers at the pooled output and at the encoder output's other consumers
(cross-modal K/V, alignment).  The HIP path's worst audio tensor must lie within max(1e-2, that
floor's worst + 0.1 points); every other tensor within 1e-2.  Measured (round 5, profiles/
r5_parity.txt): c1 1.17 % vs floor 1.25 %, c2 0.87 / 0.90 %, c4 0.98 / 0.99 %, c5 1.10 / 1.02 %.
The margin is not slack for the kernels: the pooling scorer's gradients move by ±0.2 points
between runs whose forwards differ at the 1e-6 level (they difference nearly equal frames).
Over six fresh draws per config (profiles/r5_seed_sweep.jsonl), HIP-minus-floor on the worst
tensor averages +0.04 / +0.02 / -0.08 points at c1 / c2 / c5, with about 0.2 points of single-draw
noise.  At c5 the largest per-tensor excess is a distance table, a different layer each draw
(DESIGN §4).
"""
import pytest
import torch
import torch.nn.functional as F

from kref import bf16_exact_model_
from oracle import ref_model as R
import precision_probe as PP

pytestmark = pytest.mark.gpu

CONFIGS = {  # name: (batch, samples, tokens, unfreeze k, align, freeze_encoders, fp8, bf16-exact weights)
    "c1": (4, 32000, 16, 3, False, "partial", False, True),
    "c2": (2, 160000, 64, 3, False, "partial", False, True),
    "c4": (2, 160000, 64, 5, True, "partial", False, True),
    "c5": (1, 480000, 64, 3, False, "none", False, True),
    "c5_fp8": (1, 480000, 64, 3, False, "none", True, True),
    # + the Conformer input-gradient GEMMs on MX-fp8 (opt-in engine.fp8_bwd)
    "c5_fp8bwd": (1, 480000, 64, 3, False, "none", "bwd", True),
    # end to end with arbitrary fp32 master weights: the bf16 quantisation of the weights included
    "c2_fp32w": (2, 160000, 64, 3, False, "partial", False, False),
    # the bench's kernel plan: every GEMM with a 256x256 output tile on the
    # persistent 8-phase kernels (ops.bench_gemm_plan), so this B = 2 / B = 1 instance runs the
    # compile-time epilogue instantiations the b = 64 step runs (<515,1>, <516,11>, <548,11>,
    # <65,0>, <72,0>, <513,0>, <512,0> ...) and, at c5 with fp8, the 8-phase MX-fp8 kernel
    "c2_8ph": (2, 160000, 64, 3, False, "partial", False, True),
    "c5_fp8_8ph": (1, 480000, 64, 3, False, "none", True, True),
}
BENCH_PLAN = {"c2_8ph", "c5_fp8_8ph"}
# Seeded draws of (weights, clips, cotangents) per bf16-exact config: draw 0 is the original
# instance (model 0, data 3, cotangent 5); draw d >= 1 is profiles/r5_seed_sweep.py's seed d - 1
# (model 100 + d - 1, data 200 + d - 1, cotangent 300 + d - 1).
DRAWS = {"c1": 3, "c2": 3, "c4": 3, "c5": 3}
CASES = [(c, d) for c in CONFIGS for d in range(DRAWS.get(c, 1))]
EXCESS = {}   # config -> {draw: HIP's worst audio tensor minus the same-instance floor's worst}


def _seeds(draw):
    return (0, 3, 5) if draw == 0 else (100 + draw - 1, 200 + draw - 1, 300 + draw - 1)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


class _AudioTap:
    """Wraps the oracle's attentive pooling of the audio states: records the encoder output h and,
    during the oracle's backward, the cotangents at the pooled output and at h's other consumers
    (cross-modal K/V, alignment) — the inputs of the same-instance floor emulation."""

    def __init__(self):
        self.cap = {}
        self.orig = R.attentive_pooling

    def __enter__(self):
        def pool(p_, pre, h, mask):
            if pre != "audio_pooling.":
                return self.orig(p_, pre, h, mask)
            self.cap = {}
            h2 = h * 1.0   # the pooling's own view of h: its hook sees only the pooling's share
            out = self.orig(p_, pre, h2, mask)
            if h.requires_grad:
                h.register_hook(lambda g: self.cap.__setitem__("dh", g.detach().clone()))
                h2.register_hook(lambda g: self.cap.__setitem__("dh_pool", g.detach().clone()))
                out.register_hook(lambda g: self.cap.__setitem__("dpooled", g.detach().clone()))
            return out
        R.attentive_pooling = pool
        return self

    def __exit__(self, *exc):
        R.attentive_pooling = self.orig


def _floor_errs(sd, feats, acfg, trainable, cap, probe_kw=None):
    """Per-tensor error of the emulated HIP rounding (bf16-exact weights) vs the emulation in fp32,
    on this instance's audio weights, clips and oracle cotangents (probe_kw: extra rounding points
    for diagnostics, precision_probe.Probe keywords)."""
    names = [n for n in sd if n.startswith(("audio_encoder.", "audio_pooling."))]
    tr = {n for n in names if n in trainable}
    dpooled = cap["dpooled"]
    dh_other = cap["dh"] - cap["dh_pool"]
    g = {}
    for tag, fl in (("fp32", {}), ("hip", {k: k != "w" for k in PP.FLAGS})):
        pr = PP.Probe(fl, **(probe_kw if tag == "hip" and probe_kw else {}))
        p = {n: sd[n].clone().requires_grad_(n in tr) for n in names}
        h = pr.encoder(p, feats, acfg, acfg.layers)
        pooled = pr.pool(p, h)
        torch.autograd.backward([pooled, h], [dpooled, dh_other])
        g[tag] = {n: p[n].grad for n in tr if p[n].grad is not None}
    return {n: _rel(g["hip"][n], g["fp32"][n]) for n in g["fp32"] if g["fp32"][n].norm() > 1e-8}, g["fp32"]


def _hip_vs_oracle(cname, model_seed=0, data_seed=3, cot_seed=5):
    """The HIP path's forward + backward on random output cotangents and the oracle's on the same
    weights and inputs; returns the per-tensor gradient errors and what the floor emulation needs.
    The seeds default to the test's instance (profiles/r5_seed_sweep.py draws others).  BENCH_PLAN
    configs run the HIP side under ops.bench_gemm_plan() and record the GEMM kernels it launched."""
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import synthetic_batch
    B, N, L, k, align, freeze, fp8, exact = CONFIGS[cname]
    torch.manual_seed(model_seed)
    model = EnhancedAudioTextModel(use_word_alignment=align, text_layers_to_unfreeze=k, audio_layers_to_unfreeze=k,
                                   freeze_encoders=freeze, device="cuda", fp8_gemm=bool(fp8))
    model.fp8_bwd = fp8 == "bwd"
    if exact:
        bf16_exact_model_(model)
    model.eval()
    wav, lens, ids, mask, neg, nmask = synthetic_batch(B, N, L, device="cuda", seed=data_seed)
    from speech_transcript_embeddings_amd import ops
    T = ((1 + (N - 400) // 160) + 1) // 2
    feats, amask = ops.fbank(wav, lens, T, pad_value=1.0, mask_mode=0)
    batch = {"input_ids_pos": ids, "attention_mask_pos": mask, "input_ids_neg": neg, "attention_mask_neg": nmask,
             "input_values": feats, "attention_mask_audio": amask}
    from speech_transcript_embeddings_amd import align as A
    cap = {}
    fwd = A.align_forward

    def capture(*a, **kw):  # keep the HIP path's confidence-MLP pre-activations (its ReLU gate)
        r = fwd(*a, **kw)    # and the head's inputs as the HIP path feeds them (text fp32, audio bf16)
        cap["c1"] = a[-1]["align"]["c1"].float().cpu()
        b_, L_ = a[4], a[5]
        cap["hip_th"] = a[1][: b_ * L_].float().cpu().view(b_, L_, -1)
        cap["hip_ah"] = a[3].float().cpu().view(b_, a[6], -1)
        return r

    A.align_forward = capture
    plan = ops.bench_gemm_plan() if cname in BENCH_PLAN else None
    kernels = set()
    if plan is not None:
        plan.__enter__()
        ops.GEMM_TRACE = []
    try:
        try:
            outs = list(EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch))
        finally:
            A.align_forward = fwd
        if align:
            outs.append(model.last_alignment_scores)
        g = torch.Generator().manual_seed(cot_seed)
        cots = [torch.randn(o.shape, generator=g) for o in outs]
        torch.autograd.backward(outs, [c.cuda() for c in cots])
        torch.cuda.synchronize()
    finally:
        if plan is not None:
            kernels = {t[0] for t in ops.GEMM_TRACE}
            ops.GEMM_TRACE = None
            plan.__exit__(None, None, None)

    if freeze == "none":
        cfg = R.ModelCfg(use_word_alignment=align, text_layers_to_unfreeze=12, audio_layers_to_unfreeze=24)
    else:
        cfg = R.ModelCfg(use_word_alignment=align, text_layers_to_unfreeze=k, audio_layers_to_unfreeze=k)
    names = [n for n, _ in model.named_parameters()]
    trainable = R.trainable_names(names, cfg)
    assert trainable == {n for n, p_ in model.named_parameters() if p_.requires_grad}
    sd = {n: t.detach().float().cpu() for n, t in model.state_dict().items()}
    p = {n: sd[n].clone().requires_grad_(n in trainable) for n in names}
    bc = {kk: v.cpu() for kk, v in batch.items()}
    torch.set_num_threads(16)
    tap = _AudioTap()
    with tap:
        tpn, tnn, an, al = R.compute_pos_neg_embeddings(p, bc, cfg)
    flips = 0
    if align:
        # The confidence MLP's ReLU is a discrete gate (b*L x 384 units); pre-activations within
        # bf16 rounding of zero flip it and each flip moves a whole gradient row.  Re-run the
        # oracle with the HIP path's gate to check the backward at the rounding level (as
        # test_model_gpu.py does at mini size); the flips must be rare.
        assert _rel(model.last_alignment_scores, al) < 1e-2
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
        wla = R.word_level_alignment

        def wla_tap(*args):   # the head's inputs, for its same-instance floor (_align_floor)
            cap["wla_args"] = args
            return wla(*args)
        R.word_level_alignment = wla_tap
        try:
            with tap:
                tpn, tnn, an, al = R.compute_pos_neg_embeddings(p, bc, cfg)
        finally:
            R.F = R_F
            R.word_level_alignment = wla
        assert flips < 0.01 * gate.numel(), flips
        cap["gate"] = gate
    ref = [tpn, tnn, an] + ([al] if align else [])
    # fp8 bound (north_star states fp32 / bf16 only).  e4m3 keeps 3 mantissa bits, so
    # every forward GEMM of the 24 Conformer layers carries a few-percent quantisation error; at
    # full depth the embeddings land within 1e-1 of fp32 (measured 8.1 %; 4.4 % at mini depth)
    out_tol = 1e-1 if fp8 else 1e-2
    for name, got, want in zip(["txt_pos", "txt_neg", "aud", "align"], outs, ref):
        assert _rel(got, want) < out_tol, (name, _rel(got, want))
    torch.autograd.backward(ref, cots)
    params = dict(model.named_parameters())
    errs = []
    for n in names:
        if p[n].grad is None or p[n].grad.norm() < 1e-8:
            continue
        if n.endswith(("key.bias", "linear_k.bias")):
            continue  # a key bias shifts every score of a query row equally: its true gradient is 0
            # (the oracle's is fp32 round-off), so a relative error is meaningless there
        assert params[n].grad is not None, n
        errs.append((_rel(params[n].grad, p[n].grad), n))
    errs.sort(reverse=True)
    return dict(errs=errs, sd=sd, bc=bc, cfg=cfg, trainable=trainable, cap=tap.cap, p=p, flips=flips,
                kernels=kernels, align_cap=cap if align else None, cot_align=cots[3] if align else None)


def _align_floor(acap, cot):
    """The alignment head's bf16 floor on this instance: the head alone, on the alignment-score
    cotangent with the HIP path's ReLU gate, once in fp32 on the oracle's inputs and once with bf16
    rounding at align.py's rounding points (tests/precision_probe_align.py, all flags) on the
    inputs the HIP path actually fed it (its encoders' outputs: the bf16 audio states carry the
    audio encoder's own rounding into the head); per-tensor error of the head's parameter
    gradients."""
    import precision_probe_align as PA
    p_all, pre, th, ah, tm, am, heads = acap["wla_args"]
    g = {}
    for tag, on in (("fp32", False), ("hip", True)):
        fn = PA.probe_alignment({f: on for f in PA.FLAGS}, {"gate": acap["gate"]})
        pp = dict(p_all)
        for n in p_all:
            if n.startswith(pre):
                pp[n] = p_all[n].detach().clone().requires_grad_(True)
        ti, ai = (acap["hip_th"], acap["hip_ah"]) if on else (th.detach(), ah.detach())
        sc = fn(pp, pre, ti, ai, tm, am, heads)
        torch.autograd.backward([sc], [cot.view(sc.shape)])
        g[tag] = {n: pp[n].grad for n in pp if n.startswith(pre) and pp[n].grad is not None}
    return {n: _rel(g["hip"][n], g["fp32"][n]) for n in g["fp32"] if g["fp32"][n].norm() > 1e-8}


# the 8-phase instantiations a bench-plan instance must have launched (the c2 step's hot epilogues)
BENCH_KERNELS = {
    "c2_8ph": {"gemm_8ph_kernel<true, true, 515, 1>", "gemm_8ph_kernel<true, true, 516, 11>",
               "gemm_8ph_kernel<true, true, 548, 11>", "gemm_8ph_kernel<true, true, 65, 0>",
               "gemm_8ph_kernel<true, true, 64, 0>", "gemm_8ph_kernel<true, true, 513, 0>",
               "gemm_8ph_kernel<true, true, 512, 0>"},   # eval mode: the pointwise conv 2 has no dropout (<64,0>)
    "c5_fp8_8ph": {"gemm_8ph_kernel<mx8>", "gemm_8ph_kernel<true, true, 548, 11>",
                   "gemm_8ph_kernel<true, true, 512, 0>"},
}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cname,draw", CASES, ids=[f"{c}-d{d}" if DRAWS.get(c, 1) > 1 else c for c, d in CASES])
def test_full_size_vs_oracle(cname, draw):
    B, N, L, k, align, freeze, fp8, exact = CONFIGS[cname]
    r = _hip_vs_oracle(cname, *_seeds(draw))
    errs, sd, bc, cfg, trainable, p, flips = (r[x] for x in ("errs", "sd", "bc", "cfg", "trainable", "p", "flips"))
    assert len(errs) > 50
    median = errs[len(errs) // 2][0]
    tag = f"{cname} draw {draw}" if DRAWS.get(cname, 1) > 1 else cname
    print(f"[{tag}] grad rel err ({'bf16-exact' if exact else 'fp32 master'} weights): worst {errs[:6]}, "
          f"median {median:.2e}, n={len(errs)}, gate flips {flips}")
    if cname in BENCH_PLAN:
        print(f"[{tag}] GEMM kernels launched: {sorted(r['kernels'])}")
        # (the feature projection's K = 160 GEMMs stay on the 128x128 kernel, as in the bench step)
        missing = BENCH_KERNELS[cname] - r["kernels"]
        assert not missing, (missing, sorted(r["kernels"]))
    if fp8 == "bwd":
        # MX-fp8 forward AND input-gradient GEMMs (dY and Wᵀ in e4m3 with 32-k block scales; the
        # weight gradients bf16): the backward's own e4m3 rounding of every layer's dY compounds
        # over 24 layers — measured median 14.5 %, worst 34.5 % against the forward-only fp8's
        # 12 % / 29 % (profiles/r5o_fullsize.log; north_star states no fp8 bound)
        print(f"[{cname}] fp8 backward: median {median:.3f}, worst {errs[0][0]:.3f}")
        assert median < 2e-1 and errs[0][0] < 4.5e-1, (median, errs[:5])
    elif fp8:
        # elementwise vs fp32 with fp8-quantised forward activations (straight-through bf16
        # backward): measured median 12 %, worst 26 % (bf16 c5: 0.7 % / 2.1 %)
        assert median < 2e-1 and errs[0][0] < 4e-1, (median, errs[:5])
    elif exact:
        # the kernels' arithmetic on bf16-exact weights against the bf16 floor of THIS instance
        # (module docstring): every tensor within north_star's 1e-2, except that an audio tensor
        # may sit where the emulated HIP rounding of the same weights, clips and cotangents puts
        # the worst one, + 0.1 points
        floor, g_emul = _floor_errs(sd, bc["input_values"], cfg.audio, trainable, r["cap"])
        # the emulation in fp32 is the oracle's own audio backward (same cotangents): a check
        # that the floor was measured on the graph the oracle differentiates
        emul_err = max(_rel(g_emul[n], p[n].grad) for n in g_emul
                       if not n.endswith(("linear_k.bias", "attention.2.bias")))   # true gradient 0
        fl = sorted(((e, n) for n, e in floor.items() if not n.endswith(("linear_k.bias", "attention.2.bias"))),
                    reverse=True)
        # per draw: + 0.3 points over the floor (a single draw carries about +-0.2 points of
        # realisation noise, profiles/r5_seed_sweep.jsonl); the draws' MEAN excess is bounded at
        # 0.1 points by test_full_size_mean_excess
        bound_audio = max(1e-2, fl[0][0] + 3e-3)
        aud = [(e, n) for e, n in errs if n.startswith(("audio_encoder.", "audio_pooling."))]
        rest = [(e, n) for e, n in errs if not n.startswith(("audio_encoder.", "audio_pooling."))]
        excess = aud[0][0] - fl[0][0]
        EXCESS.setdefault(cname, {})[draw] = excess
        print(f"[{tag}] same-instance bf16 floor (audio, emulated): worst {fl[:4]}, median "
              f"{fl[len(fl) // 2][0]:.2e}; emulation-vs-oracle fp32 {emul_err:.1e}; audio bound {bound_audio:.4f}")
        print(f"[{tag}] HIP worst audio {aud[0][0]:.4f} ({aud[0][1]}), floor worst {fl[0][0]:.4f} ({fl[0][1]}): "
              f"excess {excess * 100:+.3f} points")
        print(f"[{tag}] HIP vs floor on HIP's worst audio tensors: "
              + ", ".join(f"{n.replace('audio_encoder.encoder.', '')} {e:.4f}/{floor.get(n, float('nan')):.4f}"
                          for e, n in aud[:8]))
        # the alignment head (c4): its tensors end a chain of ten bf16 rounding points summed over
        # a gated MLP's rows (the mini case: GPU 1.12 % against its emulated floor 1.06 %), so they
        # are bounded like the audio tensors, by the head's own emulated floor on this instance
        bound_head = 1e-2
        if align:
            hfl = sorted(((e, n) for n, e in _align_floor(r["align_cap"], r["cot_align"]).items()), reverse=True)
            bound_head = max(1e-2, hfl[0][0] + 3e-3)
            head = [(e, n) for e, n in rest if n.startswith("word_level_alignment.")]
            print(f"[{tag}] alignment head: HIP worst {head[:2]}, same-instance bf16 floor (emulated) {hfl[:2]}; "
                  f"bound {bound_head:.4f}")
            assert not head or head[0][0] < bound_head, (head[:3], hfl[:3])
            rest = [(e, n) for e, n in rest if not n.startswith("word_level_alignment.")]
        assert emul_err < 1e-4, emul_err
        assert median < 5e-3, median
        assert aud[0][0] < bound_audio, (aud[:5], fl[:5])
        assert not rest or rest[0][0] < 1e-2, rest[:5]
    else:
        # arbitrary fp32 weights: the GEMMs read their bf16 rounding.  The fp32 reference graph
        # itself, evaluated with bf16-rounded weights and nothing else changed, moves these
        # tensors by 1.33 % worst, and under bf16 autocast by 4.8 % (profiles/r4_bf16_floor.txt)
        assert median < 1e-2, median
        assert errs[0][0] < 2.5e-2, errs[:5]


@pytest.mark.parametrize("cname", [c for c in DRAWS if DRAWS[c] > 1])
def test_full_size_mean_excess(cname):
    """Over the config's seeded draws, HIP's worst audio tensor sits at the same-instance bf16
    floor on average: mean excess <= 0.1 points (each draw: <= 0.3, checked above)."""
    ex = EXCESS.get(cname, {})
    if len(ex) < DRAWS[cname]:
        pytest.skip(f"needs all {DRAWS[cname]} draws of {cname} in this session (ran {sorted(ex)})")
    mean = sum(ex.values()) / len(ex)
    print(f"[{cname}] excess over the floor per draw (points): "
          + ", ".join(f"d{d} {e * 100:+.3f}" for d, e in sorted(ex.items())) + f"; mean {mean * 100:+.3f}")
    assert mean <= 1e-3, ex
