"""Data path on the GPU: the batched raw-waveform route (waveform_collate_fn ->
to_model_batch, one fbank launch per batch) equals the reference's route (per-clip feature
extractor -> custom_collate_fn), and a ragged batch (clips and transcripts of different
lengths, padded) gives each pair the embeddings it gets alone in a batch of one: the masks
keep padding out of every kernel."""
import numpy as np
import pytest
import torch

from test_model_gpu import load, mini_model, rel

pytestmark = pytest.mark.gpu


class _Tok:
    def __call__(self, text, max_length, padding, truncation, return_tensors):
        ids = [0] + [5 + (sum(map(ord, w)) % 900) for w in text.split()][: max_length - 2] + [2]
        mask = [1] * len(ids) + [0] * (max_length - len(ids))
        ids = ids + [1] * (max_length - len(ids))
        return {"input_ids": torch.tensor([ids]), "attention_mask": torch.tensor([mask])}


SENTENCES = ["o gato subiu no telhado", "sim", "eu gostaria de um café por favor muito obrigado",
             "duas palavras"]


def _items():
    rng = np.random.default_rng(5)
    lens = [21000, 9000, 32000, 16123]  # 1.3 s, 0.56 s, 2 s, 1.0 s
    return [{"audio": {"array": (0.1 * rng.standard_normal(n)).astype(np.float32)}, "sentence": s}
            for n, s in zip(lens, SENTENCES)]


def test_batched_waveform_route_equals_reference_route():
    from speech_transcript_embeddings_amd.data import (CommonVoiceDataset, custom_collate_fn, to_model_batch,
                                                       waveform_collate_fn)
    from speech_transcript_embeddings_amd.features import SeamlessM4TFeatureExtractor
    items = _items()
    ref_ds = CommonVoiceDataset(items, _Tok(), SeamlessM4TFeatureExtractor(padding_value=1.0), max_text_length=16)
    raw_ds = CommonVoiceDataset(items, _Tok(), None, max_text_length=16, raw_audio=True)
    import random
    random.seed(0)
    a = custom_collate_fn([ref_ds[i] for i in range(len(items))])
    random.seed(0)
    b = to_model_batch(waveform_collate_fn([raw_ds[i] for i in range(len(items))]))
    for k in ("input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg"):
        assert torch.equal(a[k].cpu(), b[k].cpu()), k
    assert a["input_values"].shape == b["input_values"].shape
    assert torch.equal(a["attention_mask_audio"].cpu().long(), b["attention_mask_audio"].cpu().long())
    torch.testing.assert_close(b["input_values"].cpu(), a["input_values"].cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("tag", ["noalign", "align"])
def test_ragged_batch_matches_single_pair_batches(tag):
    from speech_transcript_embeddings_amd.data import CommonVoiceDataset, to_model_batch, waveform_collate_fn
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    meta, _ = load(tag)
    model = mini_model(meta)
    model.eval()
    items = _items()
    ds = CommonVoiceDataset(items, _Tok(), None, max_text_length=16, raw_audio=True)
    import random
    random.seed(1)
    its = [ds[i] for i in range(len(items))]
    with torch.no_grad():
        full = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, to_model_batch(waveform_collate_fn(its)))
        full_align = model.last_alignment_scores
        assert rel(full[2][0], full[2][1]) > 1e-3  # distinct pairs, distinct embeddings
        worst = 0.0
        for i, it in enumerate(its):
            one = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, to_model_batch(waveform_collate_fn([it])))
            for x, y in zip(full, one):
                e = rel(x[i:i + 1], y)
                worst = max(worst, e)
                assert e < 1e-2, (i, e)
            if full_align is not None:
                L = int(it["attention_mask_pos"].sum())
                assert rel(full_align[i, :L], model.last_alignment_scores[0, :L]) < 1e-2
    print("worst ragged-vs-single relative error:", worst)  # measured 0.0: padding never enters a valid row
