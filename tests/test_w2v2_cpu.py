"""CPU checks of the wav2vec2 raw-waveform audio encoder's boundary:
module tree / state_dict keys and shapes equal transformers' Wav2Vec2Model (so checkpoints
load strictly), the reference's freezing rules apply, the conv-stack frame arithmetic equals
transformers', and the committed golden fixture (tests/golden/make_w2v2_golden.py) reproduces
from the in-container transformers."""
import json
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

sys.path.insert(0, str(GOLDEN))


def _hf_model(cfg_kwargs=None):
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    return Wav2Vec2Model(Wav2Vec2Config(**(cfg_kwargs or {})))


def test_tree_matches_transformers_wav2vec2_base():
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    m = EnhancedAudioTextModel(audio_model_name="facebook/wav2vec2-base", audio_embedding_dim=768, device="meta")
    ours = {n[len("audio_encoder."):]: tuple(p.shape) for n, p in m.named_parameters()
            if n.startswith("audio_encoder.")}
    with torch.device("meta"):
        hf = _hf_model()
    theirs = {n: tuple(p.shape) for n, p in hf.named_parameters()}
    assert ours == theirs
    # buffers: none on either side beyond parameters (the state_dicts are the parameter sets)
    assert set(hf.state_dict()) == set(theirs)
    # q|k|v adjacency in the flat store (one fused QKV GEMM per layer)
    st = m.store
    for i in range(12):
        pre = f"audio_encoder.encoder.layers.{i}.attention."
        o = [st.slots[pre + f"{c}_proj.weight"].offset for c in "qkv"]
        assert o[1] - o[0] == o[2] - o[1] == 768 * 768


def test_partial_freezing_follows_reference():
    """ref:355-434 freeze all but the last k `encoder.layers`, keep feature_projection trainable;
    the conv feature encoder and positional conv are not touched by it (stay trainable)."""
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    m = EnhancedAudioTextModel(audio_model_name="facebook/wav2vec2-base", audio_embedding_dim=768, device="meta",
                               audio_layers_to_unfreeze=3)
    tr = {n for n, p in m.named_parameters() if p.requires_grad and n.startswith("audio_encoder.")}
    assert all(f"audio_encoder.encoder.layers.{i}.attention.q_proj.weight" not in tr for i in range(9))
    assert all(f"audio_encoder.encoder.layers.{i}.attention.q_proj.weight" in tr for i in range(9, 12))
    assert "audio_encoder.feature_extractor.conv_layers.0.conv.weight" in tr
    assert "audio_encoder.encoder.pos_conv_embed.conv.parametrizations.weight.original1" in tr
    assert "audio_encoder.feature_projection.projection.weight" in tr
    full = EnhancedAudioTextModel(audio_model_name="facebook/wav2vec2-base", audio_embedding_dim=768, device="meta",
                                  freeze_encoders="full")
    assert not any(p.requires_grad for n, p in full.named_parameters() if n.startswith("audio_encoder."))


@pytest.mark.parametrize("n", [400, 401, 1000, 16000, 16001, 160000, 159999])
def test_frame_lengths_match_transformers(n):
    from speech_transcript_embeddings_amd.modules import W2V2Config
    with torch.device("meta"):
        hf = _hf_model()
    want = int(hf._get_feat_extract_output_lengths(torch.tensor(n)))
    assert W2V2Config().frames(n)[-1] == want


def test_unsupported_variants_raise():
    from speech_transcript_embeddings_amd.modules import W2V2Config
    for kw in ({"feat_extract_norm": "layer"}, {"conv_bias": True}, {"do_stable_layer_norm": True}):
        with pytest.raises(NotImplementedError):
            W2V2Config(**kw)


def test_golden_fixture_reproduces_from_transformers():
    """The fixture is what transformers computes (forward of both cases, float64)."""
    import make_w2v2_golden as mk
    z = np.load(GOLDEN / "w2v2_golden.npz")
    m = mk.build()
    for name, case in mk.CASES.items():
        x, mask = mk.waves(case, 10 + list(mk.CASES).index(name))
        assert np.array_equal(x, z[f"{name}/wave"])
        with torch.no_grad():
            h = m(input_values=torch.from_numpy(x).double(),
                  attention_mask=None if mask is None else torch.from_numpy(mask)).last_hidden_state
        np.testing.assert_allclose(h.float().numpy(), z[f"{name}/hidden"], rtol=0, atol=1e-5)
    cfg = json.loads((GOLDEN / "w2v2_golden.json").read_text())["config"]
    assert cfg["hidden_size"] == 64 and cfg["num_conv_pos_embedding_groups"] == 2
