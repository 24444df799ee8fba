"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/, made by
tests/golden/make_golden.py from /root/reference + transformers in the build container)."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import det_init, fbank_ref, ref_model as R


# ------------------------------------------------------------------ fbank
@pytest.fixture(scope="module")
def fb():
    return np.load(GOLDEN / "fbank_golden.npz")


@pytest.mark.parametrize("case", ["2s", "odd", "short", "1p3s"])
def test_fbank_oracle_matches_reference_extractor(fb, case):
    feats, mask = fbank_ref.extract(fb[f"{case}_wave"], padding_value=1.0)
    ref_f, ref_m = fb[f"{case}_feats"], fb[f"{case}_mask"]
    assert feats.shape == ref_f.shape
    np.testing.assert_array_equal(mask, ref_m)
    np.testing.assert_allclose(feats, ref_f, atol=2e-4, rtol=0)


def test_fbank_oracle_collate_matches_reference(fb):
    items = [fbank_ref.extract(fb[f"{c}_wave"])[0] for c in fb["cases"]]
    feats, mask = fbank_ref.collate(items)
    np.testing.assert_array_equal(mask, fb["batch_mask"])
    np.testing.assert_allclose(feats, fb["batch_feats"], atol=2e-4, rtol=0)


def test_fbank_oracle_config_size_clips():
    """10 s / 30 s / odd-F / zero-segment-in-loud / silent clips (tests/golden/fbank_cases.py)
    against the reference extractor's outputs (fbank_golden_long.npz); measured <= 1.0e-4."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    from fbank_cases import LONG_CASES, long_case_wave
    z = np.load(GOLDEN / "fbank_golden_long.npz")
    items = []
    for c, _, _ in LONG_CASES:
        feats, mask = fbank_ref.extract(long_case_wave(c), padding_value=1.0)
        np.testing.assert_array_equal(mask, z[f"{c}_mask"])
        np.testing.assert_allclose(feats, z[f"{c}_feats"], atol=2e-4, rtol=0, err_msg=c)
        items.append(feats)
    _, bmask = fbank_ref.collate(items)
    np.testing.assert_array_equal(bmask, z["batch_mask"])


def test_num_stacked_frames_survey_values():
    assert fbank_ref.num_stacked_frames(32000) == 99
    assert fbank_ref.num_stacked_frames(160000) == 499
    assert fbank_ref.num_stacked_frames(480000) == 1499


# ------------------------------------------------------------------ model
def _load(tag):
    meta = json.loads((GOLDEN / f"model_golden_{tag}.json").read_text())
    return meta, np.load(GOLDEN / f"model_golden_{tag}.npz")


def oracle_params(cfg, requires_grad_names=()):
    shapes = R.param_shapes(cfg, spec_augment=False)
    vals = det_init.state_dict_values(shapes)
    return {n: torch.from_numpy(v).requires_grad_(n in requires_grad_names) for n, v in vals.items()}


def golden_batch(z):
    keys = ["input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
            "attention_mask_audio"]
    return {k: torch.from_numpy(z[k]) for k in keys}


@pytest.mark.parametrize("tag", ["noalign", "align", "nopool", "masked"])
def test_param_tree_matches_reference(tag):
    meta, _ = _load(tag)
    cfg = R.mini_cfg(meta)
    names = [n for n, _ in R.param_shapes(cfg, spec_augment=False)]
    assert names == meta["names"]
    trainable = R.trainable_names(names, cfg)
    assert sorted(trainable) == sorted(meta["trainable"])


def test_full_size_param_counts_match_reference_logs():
    """training.log:857 (877,571,651 total / 305,994,755 trainable) and :486 (368,531,075 at k=5)."""
    counts = json.loads((GOLDEN / "param_counts.json").read_text())
    for key, (align, k) in {"align=False,k=3": (False, 3), "align=True,k=3": (True, 3),
                            "align=True,k=5": (True, 5)}.items():
        cfg = R.ModelCfg(use_word_alignment=align, text_layers_to_unfreeze=k, audio_layers_to_unfreeze=k)
        shapes = R.param_shapes(cfg, spec_augment=True)
        ref = counts[key]
        assert [n for n, _ in shapes] == list(ref["shapes"])
        assert all(list(s) == ref["shapes"][n] for n, s in shapes)
        total = sum(int(np.prod(s)) for _, s in shapes)
        tr = R.trainable_names([n for n, _ in shapes], cfg)
        assert total == ref["total"]
        assert sorted(tr) == sorted(ref["trainable_names"])


@pytest.mark.parametrize("tag", ["noalign", "align", "nopool", "masked"])
def test_model_oracle_matches_reference(tag):
    meta, z = _load(tag)
    cfg = R.mini_cfg(meta)
    p = oracle_params(cfg, set(meta["trainable"]))
    batch = golden_batch(z)
    loss, s_pos, s_neg, (tpn, tnn, an, align) = R.step_loss(p, batch, cfg)
    np.testing.assert_allclose(tpn.detach().numpy(), z["txt_pos"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(tnn.detach().numpy(), z["txt_neg"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(an.detach().numpy(), z["aud"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(s_pos.detach().numpy(), z["s_pos"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(loss.item(), float(z["loss"]), rtol=1e-5)
    if "align" in z:
        np.testing.assert_allclose(align.detach().numpy(), z["align"], atol=2e-6, rtol=1e-5)
    loss.backward()
    with_grad = set(meta["with_grad"])
    for n, t in p.items():
        if n not in with_grad:
            assert t.grad is None or not t.requires_grad, n
            continue
        g = t.grad.reshape(-1).numpy()
        gn = np.linalg.norm(g.astype(np.float64))
        assert abs(gn - float(z[f"gnorm::{n}"])) <= 1e-4 * max(1.0, gn), n
        idx = det_init.sample_indices(n, g.size)
        np.testing.assert_allclose(g[idx], z[f"gsamp::{n}"], atol=1e-6, rtol=1e-4, err_msg=n)


@pytest.mark.parametrize("tag", ["noalign", "align", "nopool", "masked"])
def test_optimizer_oracle_matches_reference(tag):
    """clip_grad_norm_(1.0) + two-group AdamW at scheduler step 1 (ref:1108-1113, 1487-1541)."""
    meta, z = _load(tag)
    cfg = R.mini_cfg(meta)
    p = oracle_params(cfg, set(meta["trainable"]))
    loss, *_ = R.step_loss(p, golden_batch(z), cfg)
    loss.backward()
    grads = {n: t.grad for n, t in p.items() if t.grad is not None}
    total = float(torch.sqrt(sum((g.double() ** 2).sum() for g in grads.values())))
    np.testing.assert_allclose(total, float(z["clip_total_norm"]), rtol=1e-5)
    coef = min(1.0, 1.0 / (total + 1e-6))
    lr_enc = R.linear_warmup_lr(meta["lr"] / 50, meta["sched_step"], meta["warmup"], meta["total_steps"])
    lr_head = R.linear_warmup_lr(meta["lr"], meta["sched_step"], meta["warmup"], meta["total_steps"])
    np.testing.assert_allclose([lr_enc, lr_head], [float(z["lr_enc"]), float(z["lr_head"])], rtol=1e-12)
    for n, g in grads.items():
        lr = lr_enc if ("text_encoder" in n or "audio_encoder" in n) else lr_head
        pn, _, _ = R.adamw_step(p[n].detach(), g * coef, torch.zeros_like(g), torch.zeros_like(g), lr=lr, step=1)
        idx = det_init.sample_indices(n, pn.numel())
        # analytically-zero gradient entries (attention key biases: softmax shift invariance) are
        # rounding noise that Adam normalises to ±lr, so for them only the bound is reproducible.
        noise = np.abs(z[f"gsamp::{n}"]) < 1e-6
        decayed = p[n].detach().reshape(-1).numpy()[idx] * (1 - lr * 0.01)
        assert np.all(np.abs(z[f"pnew::{n}"][noise] - decayed[noise]) <= lr * 1.001 + 1e-7), n
        np.testing.assert_allclose(pn.reshape(-1).numpy()[idx][~noise], z[f"pnew::{n}"][~noise], atol=1e-6,
                                   rtol=1e-5, err_msg=n)


def _infer_golden():
    meta = json.loads((GOLDEN / "infer_golden.json").read_text())
    z = np.load(GOLDEN / "infer_golden.npz")
    return meta, z


def infer_cfgs(meta):
    """(TextCfg, AudioCfg) of the inference-variant golden (RoBERTa / w2v-bert at mini dims)."""
    tx, au = meta["text"], meta["audio"]
    t = R.TextCfg(hidden=tx["hidden_size"], layers=tx["num_hidden_layers"], heads=tx["num_attention_heads"],
                  inter=tx["intermediate_size"], vocab=tx["vocab_size"], max_pos=tx["max_position_embeddings"],
                  pad_id=tx["pad_token_id"])
    a = R.AudioCfg(hidden=au["hidden_size"], layers=au["num_hidden_layers"], heads=au["num_attention_heads"],
                   inter=au["intermediate_size"], feat_in=au["feature_projection_input_dim"],
                   left=au["left_max_position_embeddings"], right=au["right_max_position_embeddings"],
                   conv_k=au["conv_depthwise_kernel_size"])
    return t, a


def test_infer_oracle_matches_golden():
    """oracle/ref_infer.py (model.py:131-329 restated) against the real model.py's outputs."""
    from oracle import ref_infer
    meta, z = _infer_golden()
    vals = det_init.state_dict_values([(n, tuple(s)) for n, s in meta["shapes"].items()])
    p = {n: torch.from_numpy(v) for n, v in vals.items()}
    batch = {k: torch.from_numpy(z[k]) for k in ("input_ids", "attention_mask", "input_features",
                                                 "attention_mask_audio")}
    t, a = infer_cfgs(meta)
    te, ae = ref_infer.forward(p, batch, t, a)
    np.testing.assert_allclose(te.numpy(), z["text_emb"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(ae.numpy(), z["audio_emb"], atol=2e-6, rtol=1e-5)
    tp, th = ref_infer.encode_text(p, batch["input_ids"], batch["attention_mask"], t)
    np.testing.assert_allclose(th.numpy(), z["text_hidden"], atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(tp.numpy(), z["text_proj"], atol=2e-5, rtol=1e-5)
