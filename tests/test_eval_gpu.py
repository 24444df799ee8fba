"""Forward-only evaluation: the reference's evaluate() loop
(trainer_unfreeze.py:1165-1284) on the HIP path.

* no_grad embeddings (engine.forward(save=False): no saved activations, FFN GEMMs without the
  pre-activation copy, attention PV on bf16 P instead of the hi/lo split the backward needs)
  match the autograd path's within 5e-3 relative and the reference's golden embeddings / loss
  (same 2e-2 bound as test_model_gpu.py);
* evaluate() returns the reference's metric keys, computed from the golden s_pos / s_neg with
  the reference's formulas (to_human_readable prob scale, mean / median / std, size-weighted
  loss), over a loader with a None batch (skipped, as in the reference);
* a forward-only pass at a long audio batch keeps far less memory alive than one that saves
  for backward."""
import numpy as np
import pytest
import torch

from test_model_gpu import batch_of, load, mini_model, rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["noalign", "align"])
def test_no_grad_embeddings_match_autograd_path_and_golden(tag):
    meta, z = load(tag)
    model = mini_model(meta)
    model.eval()
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    batch = batch_of(z)
    with torch.enable_grad():
        g_out = [t.detach().clone() for t in EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)]
        g_align = None if model.last_alignment_scores is None else model.last_alignment_scores.detach().clone()
    with torch.no_grad():
        n_out = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
        n_align = model.last_alignment_scores
    assert not any(t.requires_grad for t in n_out)
    for a, b in zip(g_out, n_out):
        assert rel(b, a.cpu().numpy()) < 5e-3
    if g_align is not None:
        assert rel(n_align, g_align.cpu().numpy()) < 5e-3
    for name, t in zip(["txt_pos", "txt_neg", "aud"], n_out):
        assert rel(t, z[name]) < 1e-2, name


@pytest.mark.parametrize("tag", ["noalign", "align"])
def test_evaluate_metrics_match_reference_formulas(tag):
    meta, z = load(tag)
    model = mini_model(meta)
    from speech_transcript_embeddings_amd.evaluate import EvalStep, evaluate, to_human_readable
    from speech_transcript_embeddings_amd.model import AlignmentAwareInfoNCE
    keys = ["input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
            "attention_mask_audio"]
    cpu_batch = {k: torch.from_numpy(z[k]) for k in keys}
    loader = [cpu_batch, None, cpu_batch]  # host tensors, moved by evaluate(); None is skipped
    loss_fn = AlignmentAwareInfoNCE(temperature=0.1, alignment_weight=0.5)
    metrics, sims = evaluate(model, loader, loss_fn, "cuda", epoch=1)
    assert not model.training
    # the reference's own formulas on its golden s_pos / s_neg / loss (two identical batches)
    sp = np.concatenate([z["s_pos"], z["s_pos"]]).astype(np.float64)
    sn = np.concatenate([z["s_neg"], z["s_neg"]]).astype(np.float64)
    clean = 1.0 / (1.0 + np.exp(-sp / 0.1))
    corrupt = 1.0 / (1.0 + np.exp(-sn / 0.1))
    want = {"loss": float(z["loss"]), "avg_similarity": clean.mean(), "median_similarity": np.median(clean),
            "std_similarity": clean.std(), "clean_similarity": clean.mean(), "corrupt_similarity": corrupt.mean(),
            "similarity_gap": clean.mean() - corrupt.mean()}
    assert set(metrics) == set(want)
    for k, v in want.items():
        # s = cos/τ with τ = 0.1 scales a bf16-level embedding error by 10 inside the sigmoid
        assert abs(float(metrics[k]) - v) <= 2e-2 * max(1.0, abs(v)), (k, metrics[k], v)
    assert len(sims) == 2 * z["s_pos"].shape[0]
    # EvalStep's s_pos is the fp32-MFMA dot product of the normalised embeddings
    batch = batch_of(z)
    sp_d, sn_d, lo_d = EvalStep(model, 0.1, 0.5)(batch)
    assert rel(sp_d, z["s_pos"]) < 2e-2 and rel(sn_d, z["s_neg"]) < 2e-2
    assert rel(lo_d[0].item(), float(z["loss"])) < 2e-2
    assert torch.allclose(to_human_readable(sp_d), torch.sigmoid(sp_d / 0.1))
    assert torch.allclose(to_human_readable(sp_d, scale="0to1"), (sp_d + 1) / 2)
    # a generic loss callable receives (s_pos, s_neg, alignment_scores=...) as in the reference
    seen = {}

    def plain_loss(s_pos, s_neg, alignment_scores=None):
        seen["align"] = alignment_scores
        return (s_pos - s_neg).mean()

    m2, _ = evaluate(model, [cpu_batch], plain_loss, "cuda")
    assert abs(m2["loss"] - float((z["s_pos"] - z["s_neg"]).mean())) < 2e-2
    assert (seen["align"] is not None) == bool(meta["use_word_alignment"])


def test_evaluate_empty_loader():
    meta, _ = load("noalign")
    model = mini_model(meta)
    from speech_transcript_embeddings_amd.evaluate import evaluate
    from speech_transcript_embeddings_amd.model import AlignmentAwareInfoNCE
    metrics, sims = evaluate(model, [None], AlignmentAwareInfoNCE(), "cuda")
    assert sims == [] and all(v == 0.0 for v in metrics.values()) and len(metrics) == 7


def test_forward_only_memory():
    """8 Conformer layers at 8 clips x 20 s (T = 999): a saving forward keeps every layer's
    activations until its outputs die; the forward-only path keeps one layer's buffers at a time."""
    import copy
    meta, _ = load("noalign")
    meta = copy.deepcopy(meta)
    meta["mini"]["audio"]["num_hidden_layers"] = 8
    model = mini_model(meta)
    model.eval()
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import synthetic_batch
    from speech_transcript_embeddings_amd import ops
    au = meta["mini"]["audio"]
    B, N, L = 8, 320000, 12
    wav, lens, ids, mask, neg, nmask = synthetic_batch(B, N, L, vocab=meta["mini"]["text"]["vocab_size"], seed=2)
    T = ((1 + (N - 400) // 160) + 1) // 2
    feats, amask = ops.fbank(wav, lens, T, pad_value=1.0, mask_mode=0)
    batch = {"input_ids_pos": ids, "attention_mask_pos": mask, "input_ids_neg": neg, "attention_mask_neg": nmask,
             "input_values": feats, "attention_mask_audio": amask}
    torch.cuda.synchronize()

    def peak(grad):
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        with torch.set_grad_enabled(grad):
            outs = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
        torch.cuda.synchronize()
        p = torch.cuda.max_memory_allocated() - base
        del outs
        return p

    p_grad, p_eval = peak(True), peak(False)
    layers = au["num_hidden_layers"]
    print(f"peak bytes: saving forward {p_grad / 2**20:.1f} MiB, forward-only {p_eval / 2**20:.1f} MiB, {layers} layers")
    assert p_eval < 0.6 * p_grad
