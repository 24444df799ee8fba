"""Data path on the CPU: transcript corruption against the reference's own
outputs (tests/golden/corruption_golden.json, made by tests/golden/make_corruption_golden.py
from trainer_unfreeze.py:784-829), the dataset wrapper's item schema, the raw-waveform collate
and the length-bucketed batch sampler."""
import json
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def test_corruption_matches_reference_golden():
    from speech_transcript_embeddings_amd.data import create_corrupted_transcript
    cases = json.loads((GOLDEN / "corruption_golden.json").read_text())["cases"]
    assert len(cases) == 320
    kinds = set()
    for c in cases:
        random.seed(c["seed"])
        out = create_corrupted_transcript(c["text"])
        assert out == c["out"], c
        assert random.random() == c["next_random"], c  # same number of draws as the reference
        if out != c["text"]:
            kinds.add(len(out.split()) - len(c["text"].split()))
    assert {-1, 0, 1} <= kinds  # drop, replace/shuffle, add all exercised (partial: < -1)


class _Tok:
    """Stand-in with the HF tokenizer call shape the reference uses (ref:836-848)."""

    def __call__(self, text, max_length, padding, truncation, return_tensors):
        assert padding == "max_length" and truncation and return_tensors == "pt"
        ids = [0] + [5 + (hash(w) % 900) for w in text.split()][: max_length - 2] + [2]
        mask = [1] * len(ids) + [0] * (max_length - len(ids))
        ids = ids + [1] * (max_length - len(ids))
        return {"input_ids": torch.tensor([ids]), "attention_mask": torch.tensor([mask])}


class _Fe:
    def __call__(self, speech, sampling_rate, return_tensors):
        n = len(speech)
        T = max(1, n // 320)
        return {"input_features": torch.full((1, T, 160), float(n)), "attention_mask": torch.ones(1, T, dtype=torch.long)}


def _items(n=7, seed=0):
    rng = np.random.default_rng(seed)
    return [{"audio": {"array": rng.standard_normal(int(rng.integers(8000, 60000))).astype(np.float32)},
             "sentence": "o gato subiu no telhado ontem"} for _ in range(n)]


def test_dataset_items_and_collates():
    from speech_transcript_embeddings_amd.data import CommonVoiceDataset, custom_collate_fn, waveform_collate_fn
    items = _items()
    ds = CommonVoiceDataset(items, _Tok(), _Fe(), max_text_length=16)
    it = ds[0]
    assert set(it) == {"input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
                       "attention_mask_audio"}
    assert it["input_ids_pos"].shape == (16,) and it["input_values"].shape[1] == 160
    b = custom_collate_fn([ds[i] for i in range(3)] + [None])
    assert b["input_values"].shape[0] == 3 and b["is_corrupted"].tolist() == [0, 0, 0]
    raw = CommonVoiceDataset(items, _Tok(), None, max_text_length=16, raw_audio=True)
    r = raw[1]
    assert "input_values" not in r and torch.equal(r["waveform"], torch.from_numpy(items[1]["audio"]["array"]))
    wb = waveform_collate_fn([raw[i] for i in range(4)] + [None])
    lens = [len(items[i]["audio"]["array"]) for i in range(4)]
    assert wb["lengths"].tolist() == lens and wb["waveform"].shape == (4, max(lens))
    for i, n in enumerate(lens):
        assert torch.equal(wb["waveform"][i, :n], torch.from_numpy(items[i]["audio"]["array"]))
        assert not wb["waveform"][i, n:].any()
    assert waveform_collate_fn([None]) is None
    with pytest.raises(ValueError):
        CommonVoiceDataset(items, _Tok(), None)


def test_length_bucket_sampler():
    from speech_transcript_embeddings_amd.data import LengthBucketBatchSampler
    rng = np.random.default_rng(3)
    lengths = (rng.lognormal(np.log(5 * 16000), 0.4, size=1000)).astype(np.int64)  # Common-Voice-like
    s = LengthBucketBatchSampler(lengths, 32, pool_batches=8, seed=7)
    batches = list(s)
    assert len(batches) == len(s) == 32
    flat = sorted(i for b in batches for i in b)
    assert flat == list(range(1000))

    def padded_fraction(bs):
        tot = sum(len(b) * lengths[b].max() for b in bs)
        return 1.0 - lengths.sum() / tot

    rand = [list(range(i, min(i + 32, 1000))) for i in range(0, 1000, 32)]
    perm = np.random.default_rng(1).permutation(1000)
    rand = [perm[b].tolist() for b in rand]
    assert padded_fraction(batches) < 0.4 * padded_fraction(rand)  # measured 0.187 vs 0.525
    assert [b for b in LengthBucketBatchSampler(lengths, 32, pool_batches=8, seed=7)] == batches  # deterministic
    s.set_epoch(1)
    assert list(s) != batches
    d = LengthBucketBatchSampler(lengths, 32, pool_batches=8, drop_last=True)
    assert all(len(b) == 32 for b in d) and len(d) == len(list(d))
