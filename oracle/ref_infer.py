"""ORACLE — test infrastructure, NOT product code (see oracle/ref_model.py's header).

CPU fp32 restatement of the reference's INFERENCE model variant, /root/reference/model.py:131-329
(EnhancedAudioTextModel as used by inference.py:48-120): RoBERTa text encoder + w2v-bert audio
encoder, attentive pooling, EnhancedProjection, and cross-modal attention whose keys/values
come straight from the encoder hidden states (no *_seq_to_projection layers, model.py:290-302),
then fusion Linear + LayerNorm and L2 normalisation (model.py:304-329).

Pinned against the reference itself: tests/golden/make_infer_golden.py runs the real model.py
and commits its outputs; tests/test_oracle_golden.py::test_infer_oracle_matches_golden checks this.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle.ref_model import (AudioCfg, TextCfg, _lin, _ln, attentive_pooling, audio_encoder, cross_modal_attention,
                              enhanced_projection, text_encoder)

XATTN_HEADS = 8  # model.py CrossModalAttention(num_heads=8)


def encode_text(p, ids, mask, tcfg: TextCfg):
    """model.py:187-199 (attentive pooling)."""
    h = text_encoder(p, ids, mask, tcfg)
    return enhanced_projection(p, "text_projection.", attentive_pooling(p, "text_pooling.", h, mask)), h


def encode_audio(p, feats, mask, acfg: AudioCfg):
    """model.py:201-246 (attentive pooling)."""
    h = audio_encoder(p, feats, mask, acfg)
    return enhanced_projection(p, "audio_projection.", attentive_pooling(p, "audio_pooling.", h, mask)), h


def forward(p, batch, tcfg: TextCfg, acfg: AudioCfg, use_cross_modal=True):
    """model.py:304-329 -> (text_embeddings, audio_embeddings), both L2-normalised."""
    tp, th = encode_text(p, batch["input_ids"], batch["attention_mask"], tcfg)
    ap, ah = encode_audio(p, batch["input_features"], batch["attention_mask_audio"], acfg)
    if use_cross_modal:  # model.py:248-277: K/V from the hidden states themselves
        t_att = cross_modal_attention(p, "text_to_audio_attention.", tp.unsqueeze(1), ah, batch["attention_mask_audio"],
                                      XATTN_HEADS).squeeze(1)
        a_att = cross_modal_attention(p, "audio_to_text_attention.", ap.unsqueeze(1), th, batch["attention_mask"],
                                      XATTN_HEADS).squeeze(1)
        tp = _ln(p, "text_fusion.1", _lin(p, "text_fusion.0", torch.cat([tp, t_att], 1)))
        ap = _ln(p, "audio_fusion.1", _lin(p, "audio_fusion.0", torch.cat([ap, a_att], 1)))
    return F.normalize(tp, p=2, dim=1), F.normalize(ap, p=2, dim=1)
