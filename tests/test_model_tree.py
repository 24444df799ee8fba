"""CPU checks of the drop-in boundary: the model's module tree, state_dict keys, shapes,
freezing rules and optimizer grouping equal the reference's (param_counts.json was
produced from the real reference model by tests/golden/make_golden.py)."""
import json

import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def counts():
    return json.loads((GOLDEN / "param_counts.json").read_text())


@pytest.mark.parametrize("key,align,k", [("align=False,k=3", False, 3), ("align=True,k=3", True, 3),
                                         ("align=True,k=5", True, 5)])
def test_full_size_tree_matches_reference(counts, key, align, k):
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    ref = counts[key]
    m = EnhancedAudioTextModel(use_word_alignment=align, text_layers_to_unfreeze=k, audio_layers_to_unfreeze=k,
                               device="meta")
    shapes = {n: list(p.shape) for n, p in m.named_parameters()}
    assert list(shapes) == list(ref["shapes"])
    assert shapes == ref["shapes"]
    assert sum(p.numel() for p in m.parameters()) == ref["total"]
    tr = [n for n, p in m.named_parameters() if p.requires_grad]
    assert sorted(tr) == sorted(ref["trainable_names"])
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == ref["trainable"]
    # flat store: gradient-receiving params first, encoder group then head group (ref:1496-1511)
    st = m.store
    enc = [n for n, s in st.slots.items() if s.segment == "enc"]
    head = [n for n, s in st.slots.items() if s.segment == "head"]
    assert all("text_encoder" in n or "audio_encoder" in n for n in enc)
    assert not any("text_encoder" in n or "audio_encoder" in n for n in head)
    nograd = {n for n, s in st.slots.items() if s.segment == "nograd"}
    # the pooler output is unused (no gradient); masked_spec_embed receives SpecAugment's
    # gradient in training mode (spec_augment=True, the default) and none without it
    assert nograd == {"text_encoder.pooler.dense.weight", "text_encoder.pooler.dense.bias"}
    assert st.slots["audio_encoder.masked_spec_embed"].segment == "enc"
    off = EnhancedAudioTextModel(use_word_alignment=align, text_layers_to_unfreeze=k, audio_layers_to_unfreeze=k,
                                 device="meta", spec_augment=False).store
    assert off.slots["audio_encoder.masked_spec_embed"].segment == "nograd"
    # fused q/k/v adjacency
    for i in range(24):
        pre = f"audio_encoder.encoder.layers.{i}.self_attn."
        o = [st.slots[pre + f"linear_{c}.weight"].offset for c in "qkv"]
        assert o[1] - o[0] == o[2] - o[1] == 1024 * 1024


def test_forward_requires_gpu_tensors():
    """No CPU fallback: the product path refuses host tensors."""
    import torch
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    m = EnhancedAudioTextModel(device="meta")
    batch = {k: torch.zeros(1, 4, dtype=torch.long) for k in
             ("input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "attention_mask_audio")}
    batch["input_values"] = torch.zeros(1, 4, 160)
    with pytest.raises(RuntimeError):
        EnhancedAudioTextModel.compute_pos_neg_embeddings(m, batch)
    with pytest.raises(ValueError):
        m({"input_values": batch["input_values"]})


@pytest.mark.parametrize("tag", ["noalign", "align", "nopool"])
def test_mini_tree_matches_reference(tag):
    """Mini-dim trees (incl. use_attentive_pooling=False: no *_pooling modules, ref:480-482)
    have the reference's state_dict keys and trainable set (model_golden_<tag>.json)."""
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.modules import AudioConfig, TextConfig
    meta = json.loads((GOLDEN / f"model_golden_{tag}.json").read_text())
    mm = meta["mini"]
    au, tx = mm["audio"], mm["text"]
    acfg = AudioConfig(hidden_size=au["hidden_size"], num_hidden_layers=au["num_hidden_layers"],
                       num_attention_heads=au["num_attention_heads"], intermediate_size=au["intermediate_size"],
                       mask_time_prob=0.0, layerdrop=0.0)
    tcfg = TextConfig(vocab_size=tx["vocab_size"], hidden_size=tx["hidden_size"],
                      num_hidden_layers=tx["num_hidden_layers"], num_attention_heads=tx["num_attention_heads"],
                      intermediate_size=tx["intermediate_size"])
    m = EnhancedAudioTextModel(text_model_name=tcfg, audio_model_name=acfg, projection_dim=mm["projection_dim"],
                               text_embedding_dim=tx["hidden_size"], audio_embedding_dim=au["hidden_size"],
                               use_word_alignment=meta["use_word_alignment"],
                               use_attentive_pooling=meta.get("use_attentive_pooling", True),
                               text_layers_to_unfreeze=mm["unfreeze"], audio_layers_to_unfreeze=mm["unfreeze"],
                               device="meta")
    assert list(m.state_dict().keys()) == meta["names"]
    assert sorted(n for n, p in m.named_parameters() if p.requires_grad) == sorted(meta["trainable"])
