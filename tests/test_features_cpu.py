"""Host-side pieces of the audio front end (features.py): frame counts and the reference's
collate semantics (ref:training/trainer_unfreeze.py:880-921).  Checked against the golden
fbank fixture's shapes (tests/golden/fbank_golden.npz, made by the real extractor)."""
import numpy as np
import torch

from conftest import GOLDEN
from speech_transcript_embeddings_amd.features import custom_collate_fn, num_frames


def test_num_frames_matches_extractor():
    assert [num_frames(n) for n in (32000, 160000, 480000)] == [99, 499, 1499]
    assert num_frames(399) == 0 and num_frames(400) == 1 and num_frames(719) == 1 and num_frames(720) == 2
    z = np.load(GOLDEN / "fbank_golden.npz")
    for c in z["cases"]:
        assert num_frames(z[f"{c}_wave"].size) == z[f"{c}_feats"].shape[0], c


def test_collate_semantics():
    items = []
    for i, (L, T) in enumerate([(5, 7), (3, 4), (6, 2)]):
        items.append({"input_ids_pos": torch.arange(1, L + 1), "attention_mask_pos": torch.ones(L, dtype=torch.long),
                      "input_ids_neg": torch.arange(10, 10 + L), "attention_mask_neg": torch.ones(L, dtype=torch.long),
                      "input_values": torch.full((T, 160), float(i + 1)), "attention_mask_audio": None})
    b = custom_collate_fn(items + [None])
    assert b["input_ids_pos"].shape == (3, 6) and b["input_ids_pos"][1, 3:].eq(0).all()
    assert b["attention_mask_neg"].sum(1).tolist() == [5, 3, 6]
    assert b["input_values"].shape == (3, 7, 160)
    assert b["input_values"][1, 4:].eq(0).all() and b["input_values"][1, :4].eq(2).all()
    assert b["attention_mask_audio"].sum(1).tolist() == [7, 4, 2]
    assert b["attention_mask_audio"].dtype == torch.long and b["is_corrupted"].tolist() == [0, 0, 0]
    assert custom_collate_fn([None]) is None
