"""wav2vec2 raw-waveform audio encoder on the HIP kernels vs transformers' Wav2Vec2Model
(SURVEY §8f rank 4).

* mini dims: against the committed float64 golden (tests/golden/make_w2v2_golden.py): hidden
  states and every parameter gradient of Σ(hidden·cot), with and without a sample mask;
* base dims (hidden 768, 12 heads, 512-channel conv stack, 128-tap / 16-group positional conv,
  2 layers, 1 s clips): against transformers run live in fp32 on the same GPU with the same
  weights — the full-size shapes of every kernel and strided GEMM view;
* a training step (TrainStep.step_batch) on raw waveforms.
Tolerances: bf16 MFMA operands with fp32 accumulation through conv stack + layers; relative L2
error per tensor (stated per assert)."""
import json
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
sys.path.insert(0, str(GOLDEN))

HID_TOL = 2e-2     # relative L2 error of last_hidden_state
GRAD_TOL = 5e-2    # relative L2 error of each parameter gradient
# The key-projection bias has an exactly zero gradient (it shifts every score of a query by the
# same q·b_k, which softmax ignores): both sides hold rounding noise, so it is checked against
# the scale of its sibling (value bias) gradient instead of relatively.
ZERO_GRAD = "attention.k_proj.bias"
ZERO_TOL = 1e-2


def _grad_errors(ours, ref):
    """{name: error} for every parameter; relative L2, or for ZERO_GRAD ‖ours‖/‖v_proj.bias grad‖."""
    errs = {}
    for n, r in ref.items():
        if n.endswith(ZERO_GRAD):
            sib = ref[n.replace("k_proj", "v_proj")]
            errs[n] = float(np.linalg.norm(ours[n]) / max(np.linalg.norm(sib), 1e-30)) * (GRAD_TOL / ZERO_TOL)
        else:
            errs[n] = _rel(ours[n], r)
    return errs


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _model(cfg):
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.modules import TextConfig
    tc = TextConfig(vocab_size=512, hidden_size=64, num_hidden_layers=1, num_attention_heads=1, intermediate_size=128,
                    max_position_embeddings=66)
    d = cfg.hidden_size
    m = EnhancedAudioTextModel(text_model_name=tc, audio_model_name=cfg, projection_dim=64, text_embedding_dim=64,
                               audio_embedding_dim=d, freeze_encoders=False, spec_augment=False, device="cuda")
    return m.train()


def _mini():
    from speech_transcript_embeddings_amd.modules import W2V2Config
    cfg = json.loads((GOLDEN / "w2v2_golden.json").read_text())["config"]
    return W2V2Config(**cfg)


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN / "w2v2_golden.npz")


@pytest.mark.parametrize("case", ["mask", "nomask"])
def test_mini_matches_transformers_golden(golden, case):
    m = _model(_mini())
    sd = {k[len("param/"):]: torch.from_numpy(golden[k]) for k in golden.files if k.startswith("param/")}
    m.audio_encoder.load_state_dict(sd, strict=True)
    wave = torch.from_numpy(golden[f"{case}/wave"]).cuda()
    mask = torch.from_numpy(golden[f"{case}/mask"]).cuda() if f"{case}/mask" in golden.files else None
    m.zero_grad(set_to_none=True)
    _, hidden = m.encode_audio(wave, mask)
    ref_h = golden[f"{case}/hidden"]
    assert hidden.shape == ref_h.shape
    e_h = _rel(hidden.detach().cpu().numpy(), ref_h)
    assert e_h < HID_TOL, e_h
    cot = torch.from_numpy(golden[f"{case}/cot"]).cuda()
    (hidden * cot).sum().backward()
    torch.cuda.synchronize()
    params = dict(m.audio_encoder.named_parameters())
    pre = f"{case}/grad/"
    ref = {k[len(pre):]: golden[k] for k in golden.files if k.startswith(pre)}
    assert all(params[n].grad is not None for n in ref)
    errs = _grad_errors({n: params[n].grad.cpu().numpy() for n in ref}, ref)
    bad = {n: e for n, e in errs.items() if not e < GRAD_TOL}
    assert not bad, bad
    assert len(errs) == len(params)


def test_base_dims_match_transformers_live():
    """wav2vec2-base shapes (2 layers) against transformers fp32 on the GPU, same weights."""
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    from speech_transcript_embeddings_amd.modules import W2V2Config
    kw = dict(num_hidden_layers=2, hidden_dropout=0.0, activation_dropout=0.0, attention_dropout=0.0,
              feat_proj_dropout=0.0, layerdrop=0.0, mask_time_prob=0.0)
    torch.manual_seed(0)
    hf = Wav2Vec2Model(Wav2Vec2Config(**kw, attn_implementation="eager")).cuda().train()
    with torch.no_grad():
        g = torch.Generator(device="cuda").manual_seed(1)
        for n, p in hf.named_parameters():
            if n.endswith("bias"):
                p.copy_(0.1 * torch.randn(p.shape, device="cuda", generator=g))
    m = _model(W2V2Config(**kw))
    m.audio_encoder.load_state_dict({k: v.detach().float() for k, v in hf.state_dict().items()}, strict=True)
    B, N = 2, 16000
    gen = torch.Generator(device="cuda").manual_seed(2)
    wave = torch.randn(B, N, device="cuda", generator=gen)
    mask = torch.ones(B, N, dtype=torch.int64, device="cuda")
    mask[1, 11000:] = 0
    wave[1, 11000:] = 0
    ref = hf(input_values=wave, attention_mask=mask).last_hidden_state
    _, hid = m.encode_audio(wave, mask)
    assert hid.shape == ref.shape
    e_h = _rel(hid.detach().cpu().numpy(), ref.detach().cpu().numpy())
    assert e_h < HID_TOL, e_h
    cot = torch.randn(ref.shape, device="cuda", generator=gen)
    (ref * cot).sum().backward()
    m.zero_grad(set_to_none=True)
    (hid * cot).sum().backward()
    ours = dict(m.audio_encoder.named_parameters())
    ref = {n: p.grad.cpu().numpy() for n, p in hf.named_parameters() if p.grad is not None}
    errs = _grad_errors({n: ours[n].grad.cpu().numpy() for n in ref}, ref)
    bad = {n: e for n, e in errs.items() if not e < GRAD_TOL}
    assert not bad, bad


def test_train_step_on_raw_waveforms():
    """TrainStep on a wav2vec2 model: raw samples in, finite loss, finite non-zero gradients down to
    the first conv layer, and an optimizer step that moves the weights (second step: the linear
    warmup's first factor is 0, as in the reference's scheduler)."""
    from speech_transcript_embeddings_amd.train import TrainStep
    m = _model(_mini())
    step = TrainStep(m, gather_embeddings=False)
    B, N, L = 4, 4000, 12
    g = torch.Generator(device="cuda").manual_seed(3)
    wav = torch.randn(B, N, device="cuda", generator=g)
    lengths = torch.tensor([4000, 3500, 3000, 2600], device="cuda", dtype=torch.int32)
    ids = torch.randint(3, 500, (B, L), device="cuda", generator=g)
    am = torch.ones(B, L, dtype=torch.int64, device="cuda")
    w0 = m.audio_encoder.feature_extractor.conv_layers[0].conv.weight.detach().clone()
    out = step(wav, lengths, ids, am, ids.flip(0), am)
    loss = float(out)
    assert np.isfinite(loss)
    g0 = m.store.g("audio_encoder.feature_extractor.conv_layers.0.conv.weight")  # the flat gradient buffer
    assert g0 is not None and torch.isfinite(g0).all() and float(g0.abs().sum()) > 0
    assert np.isfinite(float(step(wav, lengths, ids, am, ids.flip(0), am)))
    w1 = m.audio_encoder.feature_extractor.conv_layers[0].conv.weight.detach()
    assert not torch.equal(w0, w1)
    assert torch.isfinite(w1).all()
