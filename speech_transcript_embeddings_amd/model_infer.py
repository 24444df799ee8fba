"""The reference's inference model variant, forward-only on the HIP path.

/root/reference/model.py:131-329 defines a second EnhancedAudioTextModel, the one inference.py
(:48-120) loads: a RoBERTa-large text encoder (sentence-transformers/all-roberta-large-v1,
1024-d, 24 layers), w2v-bert-2.0 audio, projection_dim 1024, frozen encoders, and cross-modal
attention whose keys/values are the encoder hidden states themselves (no *_seq_to_projection
layers, model.py:248-277).  forward(batch) takes {"input_ids", "attention_mask",
"input_features", "attention_mask_audio"} and returns L2-normalised (text_embeddings,
audio_embeddings) (model.py:304-329).

Same class name, constructor, state_dict keys and methods (encode_text, encode_audio,
apply_cross_modal_attention, forward), so `model.load_state_dict(checkpoint["model_state_dict"])`
of a reference inference checkpoint works unchanged.  Every op runs on libste.so kernels: the
encoders through engine.text_forward / audio_forward (no saved activations), pooling,
projection, the single-query cross attention (xattn1) and the fusion GEMM + LayerNorm.
Inference only: there is no backward for this variant (the reference trains the other one).
"""
from __future__ import annotations

import logging

import torch
import torch.nn as nn

from . import ops
from .engine import Engine
from .model import EnhancedAudioTextModel as _TrainModel
from .model import _resolve
from .modules import (AttentivePooling, AudioConfig, AudioEncoder, CrossModalAttention, EnhancedProjection, TextConfig,
                      TextEncoder)
from .store import ParamStore

logger = logging.getLogger(__name__)
BF16, F32 = torch.bfloat16, torch.float32

# RoBERTa-large (all-roberta-large-v1's encoder: transformers RobertaConfig of roberta-large)
ROBERTA_LARGE = TextConfig(vocab_size=50265, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                           intermediate_size=4096, max_position_embeddings=514, type_vocab_size=1,
                           layer_norm_eps=1e-5, pad_token_id=1)
_TEXT_CONFIGS = {"sentence-transformers/all-roberta-large-v1": ROBERTA_LARGE, "roberta-large": ROBERTA_LARGE}
_AUDIO_CONFIGS = {"facebook/w2v-bert-2.0": AudioConfig()}


class EnhancedAudioTextModel(nn.Module):
    """model.py:131-329 (inference variant)."""

    def __init__(self, text_model_name="sentence-transformers/all-roberta-large-v1",
                 audio_model_name="facebook/w2v-bert-2.0", projection_dim=1024, text_embedding_dim=1024,
                 audio_embedding_dim=1024, dropout=0.1, use_cross_modal=True, use_attentive_pooling=True,
                 freeze_encoders=True, device="cuda"):
        super().__init__()
        self.text_cfg = _resolve(text_model_name, _TEXT_CONFIGS, TextConfig)
        self.audio_cfg = _resolve(audio_model_name, _AUDIO_CONFIGS, AudioConfig)
        if use_cross_modal and not (self.text_cfg.hidden_size == self.audio_cfg.hidden_size == projection_dim):
            raise ValueError("model.py's cross-modal attention reads the encoder hidden states directly: "
                             "text and audio hidden sizes must equal projection_dim")
        with torch.device("meta"):
            self.text_encoder = TextEncoder(self.text_cfg)
            self.audio_encoder = AudioEncoder(self.audio_cfg)
            self.projection_dim = projection_dim
            self.use_cross_modal = use_cross_modal
            self.use_attentive_pooling = use_attentive_pooling
            self.dropout = dropout
            self.xattn_heads = 8
            if freeze_encoders:
                for p in list(self.text_encoder.parameters()) + list(self.audio_encoder.parameters()):
                    p.requires_grad = False
            self.text_projection = EnhancedProjection(text_embedding_dim, projection_dim, dropout=dropout)
            self.audio_projection = EnhancedProjection(audio_embedding_dim, projection_dim, dropout=dropout)
            if use_cross_modal:
                self.text_to_audio_attention = CrossModalAttention(projection_dim, dropout=dropout)
                self.audio_to_text_attention = CrossModalAttention(projection_dim, dropout=dropout)
                self.text_fusion = nn.Sequential(nn.Linear(2 * projection_dim, projection_dim),
                                                 nn.LayerNorm(projection_dim))
                self.audio_fusion = nn.Sequential(nn.Linear(2 * projection_dim, projection_dim),
                                                  nn.LayerNorm(projection_dim))
            if use_attentive_pooling:  # else CLS text / masked-mean audio (ref model.py:214-216, 255-270)
                self.text_pooling = AttentivePooling(text_embedding_dim)
                self.audio_pooling = AttentivePooling(audio_embedding_dim)
        self.store = ParamStore(self, device, has_grad=set())  # forward only: no gradient buffer
        _TrainModel._init_params(self)
        self.store.sync_shadow(force=True)
        self.engine = Engine(self)

    # -------------------------------------------------------------- pieces
    def _text(self, input_ids, attention_mask):
        e, ctx = self.engine, {}
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        B, L = input_ids.shape
        h, hb = e.text_forward(input_ids.contiguous(), attention_mask.contiguous(), False, 0, ctx, save=False)
        pooled = e._pool_fwd("text_pooling", h, hb, ctx["t_mask32"], B, L, {})
        return e._proj_fwd("text_projection", pooled, B, False, 0, {}), h, hb, ctx["t_mask32"]

    def _audio(self, input_features, attention_mask):
        e, ctx = self.engine, {}
        B, T, _ = input_features.shape
        if attention_mask is None:
            attention_mask = torch.ones(B, T, dtype=torch.int64, device=input_features.device)
        h, hb = e.audio_forward(input_features.contiguous(), attention_mask.contiguous(), False, 0, ctx, save=False)
        pooled = e._pool_fwd("audio_pooling", h, hb, ctx["a_mask32"], B, T, {}, hs=ctx.get("a_hs"))
        return e._proj_fwd("audio_projection", pooled, B, False, 0, {}), h, hb, ctx["a_mask32"]

    def _attend(self, name, q_proj, kv_hb, mask32, B, S):
        """CrossModalAttention(q = q_proj as one token, k = v-source = kv_hb) (model.py:79-117)."""
        s, e = self.store, self.engine
        P = self.projection_dim
        kv = ops.linear(kv_hb, s.fused(name + ".key.weight", 2, "w"), s.fused(name + ".key.bias", 2, "p"),
                        out_bf16=True)
        q = ops.linear(q_proj.float().contiguous(), e._w32(name + ".query.weight"), s.p(name + ".query.bias"))
        att = e._e(B, P)
        ops.xattn1_fwd(q, kv[:, :P], kv[:, P:], mask32, B, S, self.xattn_heads, e._e(B * self.xattn_heads * S), att)
        return ops.linear(att, e._w32(name + ".out_proj.weight"), s.p(name + ".out_proj.bias"))

    def _fuse(self, name, proj, att):
        e = self.engine
        B, P = proj.shape
        cat = e._e(B, 2 * P)
        ops.copy2d(cat[:, :P], proj.float().contiguous())
        ops.copy2d(cat[:, P:], att.float().contiguous())
        return e._fuse_fwd(name, cat)[0]

    # ------------------------------------------------------------ reference API
    @torch.no_grad()
    def encode_text(self, input_ids, attention_mask=None):
        """model.py:187-199: (projection [B,P], last_hidden_state [B,L,H])."""
        self.store.sync_shadow()
        proj, h, _, _ = self._text(input_ids, attention_mask)
        return proj, h.view(input_ids.shape[0], input_ids.shape[1], -1)

    @torch.no_grad()
    def encode_audio(self, input_features, attention_mask=None):
        """model.py:201-246: (projection [B,P], last_hidden_state [B,T,H])."""
        self.store.sync_shadow()
        proj, h, _, _ = self._audio(input_features, attention_mask)
        return proj, h.view(input_features.shape[0], input_features.shape[1], -1)

    @torch.no_grad()
    def apply_cross_modal_attention(self, text_projected, text_hidden, text_mask, audio_projected, audio_hidden,
                                    audio_mask):
        """model.py:248-277 on already-encoded inputs -> (text_fused, audio_fused)."""
        if not self.use_cross_modal:
            return text_projected, audio_projected
        self.store.sync_shadow()
        e = self.engine
        B, L, H = text_hidden.shape
        T = audio_hidden.shape[1]
        thb = ops.cast_bf16(text_hidden.reshape(B * L, H).contiguous(), e._e(B * L, H, dtype=BF16))
        ahb = ops.cast_bf16(audio_hidden.reshape(B * T, H).contiguous(), e._e(B * T, H, dtype=BF16))
        tm = e._e(B * L, dtype=torch.int32)
        am = e._e(B * T, dtype=torch.int32)
        from . import _lib
        _lib.call("ste_mask_i64_to_f32", text_mask.contiguous().data_ptr(), None, tm.data_ptr(), B * L,
                  _lib.stream_ptr())
        _lib.call("ste_mask_i64_to_f32", audio_mask.contiguous().data_ptr(), None, am.data_ptr(), B * T,
                  _lib.stream_ptr())
        t_att = self._attend("text_to_audio_attention", text_projected, ahb, am, B, T)
        a_att = self._attend("audio_to_text_attention", audio_projected, thb, tm, B, L)
        return self._fuse("text_fusion", text_projected, t_att), self._fuse("audio_fusion", audio_projected, a_att)

    @torch.no_grad()
    def forward(self, batch):
        """model.py:304-329 -> (text_embeddings, audio_embeddings), L2-normalised."""
        for k in ("input_ids", "attention_mask", "input_features", "attention_mask_audio"):
            if batch[k].device.type != "cuda":
                raise RuntimeError(f"batch[{k!r}] must be on the GPU (libste.so has no CPU path)")
        self.store.sync_shadow()
        B, L = batch["input_ids"].shape
        T = batch["input_features"].shape[1]
        tproj, _, thb, tm = self._text(batch["input_ids"], batch["attention_mask"])
        aproj, _, ahb, am = self._audio(batch["input_features"], batch["attention_mask_audio"])
        if self.use_cross_modal:
            t_att = self._attend("text_to_audio_attention", tproj, ahb, am, B, T)
            a_att = self._attend("audio_to_text_attention", aproj, thb, tm, B, L)
            tproj = self._fuse("text_fusion", tproj, t_att)
            aproj = self._fuse("audio_fusion", aproj, a_att)
        te, ae = torch.empty_like(tproj), torch.empty_like(aproj)
        ops.l2norm_fwd(tproj.contiguous(), te, torch.empty(B, device=te.device))
        ops.l2norm_fwd(aproj.contiguous(), ae, torch.empty(aproj.shape[0], device=ae.device))
        return te, ae
