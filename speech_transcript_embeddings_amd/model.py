"""Drop-in replacements for the reference's model / loss API
(ref = /root/reference/training/trainer_unfreeze.py):

  EnhancedAudioTextModel   ref:315-697  (same constructor arguments, attribute tree,
                                          compute_pos_neg_embeddings, forward, last_alignment_scores)
  AlignmentAwareInfoNCE    ref:702-742  (same constructor / forward signature)

`train_epoch` (ref:1026-1162) runs unmodified on top of these: its
compute_pos_neg_embeddings -> (aud*txt).sum(1) -> loss_fn -> loss.backward() ->
clip_grad_norm_ -> optimizer.step() sequence works because the whole model forward
is ONE autograd node whose backward is the HIP schedule of engine.py and which
leaves the parameter gradients in `param.grad` (views of the flat gradient buffer).
"""
from __future__ import annotations

import logging

import torch
from torch import nn

from . import ops, torch_ops  # noqa: F401  (registers the ste:: custom ops)
from .engine import Engine
from .modules import (AttentivePooling, AudioConfig, AudioEncoder, CrossModalAttention, EnhancedProjection,
                      TextConfig, TextEncoder, W2V2AudioEncoder, W2V2Config, WordLevelAlignmentModule)
from .store import ParamStore

logger = logging.getLogger(__name__)

# encoder names the reference passes to AutoModel.from_pretrained -> architecture configs
_TEXT_CONFIGS = {
    "sentence-transformers/paraphrase-multilingual-mpnet-base-v2": TextConfig(),
    "xlm-roberta-base": TextConfig(),
}
_AUDIO_CONFIGS = {"facebook/w2v-bert-2.0": AudioConfig(),
                  # raw-waveform wav2vec2 (wav2vec2.py)
                  "facebook/wav2vec2-base": W2V2Config(), "facebook/wav2vec2-base-960h": W2V2Config(),
                  "facebook/wav2vec2-base-100h": W2V2Config()}


def _resolve(name_or_cfg, table, default_cls):
    if isinstance(name_or_cfg, (TextConfig, AudioConfig, W2V2Config)):
        return name_or_cfg
    if name_or_cfg in table:
        return table[name_or_cfg]
    logger.warning("unknown encoder name %r: using the default %s architecture (random init, no download)",
                   name_or_cfg, default_cls.__name__)
    return default_cls()


class EnhancedAudioTextModel(nn.Module):
    """ref:315-697.  Encoders are built from architecture configs (there is no
    network: weights are random-initialised or loaded with load_state_dict).
    spec_augment (default on, like the reference's w2v-bert config): SpecAugment time masking of
    the audio encoder input in training mode (specaug.py).
    fp8_gemm (BASELINE config 5, "fp8 MFMA GEMMs"; default off): the Conformer layers' forward
    nn.Linear GEMMs run MX-fp8 (e4m3 operands, E8M0 scales per 32 k; ste_gemm_mx8), gradients
    stay bf16 (straight-through: dX/dW GEMMs read the bf16 weights and saved bf16 activations)."""

    def __init__(self, text_model_name="sentence-transformers/paraphrase-multilingual-mpnet-base-v2",
                 audio_model_name="facebook/w2v-bert-2.0", projection_dim=768, text_embedding_dim=768,
                 audio_embedding_dim=1024, dropout=0.1, use_cross_modal=True, use_attentive_pooling=True,
                 use_word_alignment=False, freeze_encoders="partial", text_layers_to_unfreeze=5,
                 audio_layers_to_unfreeze=5, device="cuda", spec_augment=True, fp8_gemm=False):
        super().__init__()
        self.fp8_gemm = fp8_gemm
        self.fp8_bwd = False   # opt-in with fp8_gemm: the Conformer input-gradient GEMMs on MX-fp8 too
        self.text_cfg = _resolve(text_model_name, _TEXT_CONFIGS, TextConfig)
        self.audio_cfg = _resolve(audio_model_name, _AUDIO_CONFIGS, AudioConfig)
        with torch.device("meta"):  # no host-side weights: values are initialised in the HBM store
            self._build(projection_dim, text_embedding_dim, audio_embedding_dim, dropout, use_cross_modal,
                        use_attentive_pooling, use_word_alignment, freeze_encoders, text_layers_to_unfreeze,
                        audio_layers_to_unfreeze, spec_augment)
        has_grad = {n for n, p in self.named_parameters() if p.requires_grad}
        has_grad -= {n for n in has_grad if n.startswith("text_encoder.pooler.")}
        if not spec_augment:
            has_grad.discard("audio_encoder.masked_spec_embed")
        self.store = ParamStore(self, device, has_grad)
        self._init_params()
        self.store.sync_shadow(force=True)
        self.engine = Engine(self)
        self.last_alignment_scores = None
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        total = sum(p.numel() for p in self.parameters())
        logger.info("Model initialized with %s trainable parameters out of %s total", f"{trainable:,}",
                    f"{total:,}")

    def _build(self, projection_dim, text_embedding_dim, audio_embedding_dim, dropout, use_cross_modal,
               use_attentive_pooling, use_word_alignment, freeze_encoders, text_layers_to_unfreeze,
               audio_layers_to_unfreeze, spec_augment):
        self.text_encoder = TextEncoder(self.text_cfg)
        self.audio_encoder = (W2V2AudioEncoder if isinstance(self.audio_cfg, W2V2Config) else AudioEncoder)(
            self.audio_cfg)
        self.text_hidden_dim = self.text_cfg.hidden_size
        self.audio_hidden_dim = self.audio_cfg.hidden_size
        self.projection_dim = projection_dim
        self.use_cross_modal = use_cross_modal
        self.use_attentive_pooling = use_attentive_pooling
        self.use_word_alignment = use_word_alignment
        self.dropout = dropout
        self.xattn_heads = 8
        self.spec_augment = spec_augment
        # constructor arguments the reference's checkpoint dict records (ref:1617-1633)
        self.freeze_encoders = freeze_encoders
        self.text_layers_to_unfreeze = text_layers_to_unfreeze
        self.audio_layers_to_unfreeze = audio_layers_to_unfreeze
        self._apply_freezing(freeze_encoders, text_layers_to_unfreeze, audio_layers_to_unfreeze)
        self.text_projection = EnhancedProjection(text_embedding_dim, projection_dim, dropout=dropout)
        self.audio_projection = EnhancedProjection(audio_embedding_dim, projection_dim, dropout=dropout)
        if use_cross_modal:
            self.text_seq_to_projection = nn.Linear(self.text_hidden_dim, projection_dim)
            self.audio_seq_to_projection = nn.Linear(self.audio_hidden_dim, projection_dim)
            self.text_to_audio_attention = CrossModalAttention(projection_dim, dropout=dropout)
            self.audio_to_text_attention = CrossModalAttention(projection_dim, dropout=dropout)
            self.text_fusion = nn.Sequential(nn.Linear(2 * projection_dim, projection_dim),
                                             nn.LayerNorm(projection_dim))
            self.audio_fusion = nn.Sequential(nn.Linear(2 * projection_dim, projection_dim),
                                              nn.LayerNorm(projection_dim))
        if use_attentive_pooling:  # else CLS text / masked-mean audio, no parameters (ref:480-482)
            self.text_pooling = AttentivePooling(text_embedding_dim)
            self.audio_pooling = AttentivePooling(audio_embedding_dim)
        if use_word_alignment:
            self.word_level_alignment = WordLevelAlignmentModule(self.text_hidden_dim, self.audio_hidden_dim,
                                                                 projection_dim, dropout=dropout)

    # ref:355-434
    def _apply_freezing(self, mode, k_text, k_audio):
        if mode == "full" or mode is True:
            for p in list(self.text_encoder.parameters()) + list(self.audio_encoder.parameters()):
                p.requires_grad = False
        elif mode == "partial":
            layers = self.text_encoder.encoder.layer
            for i, layer in enumerate(layers):
                if i < len(layers) - k_text:
                    for p in layer.parameters():
                        p.requires_grad = False
            for p in self.text_encoder.pooler.parameters():
                p.requires_grad = True
            layers = self.audio_encoder.encoder.layers
            for i, layer in enumerate(layers):
                if i < len(layers) - k_audio:
                    for p in layer.parameters():
                        p.requires_grad = False
            for p in self.audio_encoder.feature_projection.parameters():
                p.requires_grad = True

    def _init_params(self, seed: int = 0):
        """Random init (no checkpoint download is possible): encoders N(0, 0.02) like the HF
        initializers, LayerNorms 1/0, heads like torch's nn.Linear defaults (xavier for the
        cross-modal attention projections, ref:121-124)."""
        if self.store.device.type == "meta":
            return
        g = torch.Generator(device=self.store.device).manual_seed(seed)
        with torch.no_grad():
            for n, p in self.named_parameters():
                leaf = n.rsplit(".", 1)[-1]
                is_norm = ("norm" in n.lower() or "LayerNorm" in n) and leaf in ("weight", "bias")
                if is_norm:
                    p.fill_(1.0 if leaf == "weight" else 0.0)
                elif n.startswith(("text_encoder", "audio_encoder")):
                    if leaf == "bias":
                        p.zero_()
                    elif n.endswith("masked_spec_embed"):
                        p.uniform_(0.0, 1.0, generator=g)
                    elif n.endswith("parametrizations.weight.original1"):
                        # wav2vec2 positional conv v (transformers' init: N(0, 2/(k·Cin/groups)))
                        p.normal_(0.0, (2.0 / (p.shape[1] * p.shape[2])) ** 0.5, generator=g)
                    elif n.endswith("parametrizations.weight.original0"):
                        pass  # g = ‖v‖ per tap, set below once v is drawn
                    elif ".conv_layers." in n and n.endswith("conv.weight"):
                        nn.init.kaiming_normal_(p, generator=g)
                    else:
                        p.normal_(0.0, 0.02, generator=g)
                elif leaf in ("in_proj_bias",) or (leaf == "bias" and "_attention" in n):
                    p.zero_() if leaf == "in_proj_bias" else p.uniform_(-p.shape[0] ** -0.5, p.shape[0] ** -0.5,
                                                                         generator=g)
                else:
                    fan_in = p.shape[-1] if p.dim() > 1 else p.shape[0]
                    fan_out = p.shape[0]
                    if "_attention." in n and leaf == "weight" or leaf == "in_proj_weight":
                        a = (6.0 / (fan_in + fan_out)) ** 0.5
                    else:
                        a = fan_in ** -0.5
                    p.uniform_(-a, a, generator=g)
            params = dict(self.named_parameters())
            for n, p in params.items():
                if n.endswith("parametrizations.weight.original0"):
                    p.copy_(params[n[:-1] + "1"].pow(2).sum(dim=(0, 1), keepdim=True).sqrt())

    # ---------------------------------------------------------------- API
    @staticmethod
    def compute_pos_neg_embeddings(model, batch):
        """ref:502-565: returns L2-normalised (txt_pos, txt_neg, aud) [B, P]; sets
        model.last_alignment_scores when use_word_alignment."""
        return model._embed(batch)

    def forward(self, batch):
        if "input_ids_pos" not in batch or "input_ids_neg" not in batch:
            raise ValueError("Batch must contain 'input_ids_pos' and 'input_ids_neg'. "
                             "Got keys: {}".format(list(batch.keys())))
        return EnhancedAudioTextModel.compute_pos_neg_embeddings(self, batch)

    def _embed(self, batch):
        for k in ("input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
                  "attention_mask_audio"):
            if k == "attention_mask_audio" and batch.get(k) is None and self.engine.raw_audio:
                continue  # wav2vec2: no sample mask = every frame valid
            if batch[k].device.type != "cuda":
                raise RuntimeError(f"batch[{k!r}] must be on the GPU (libste.so has no CPU path)")
        self.store.sync_shadow()
        if not torch.is_grad_enabled():
            # forward only (the reference's evaluate() under torch.no_grad, ref:1188-1198): no
            # autograd node, no saved activations
            tf_p, tf_n, af, align, _ = self.engine.forward(batch, self.training, save=False)
            tpn, tnn, an = _l2_normalise(tf_p, tf_n, af)[0]
            self.last_alignment_scores = align if self.use_word_alignment else None
            return tpn, tnn, an
        dummy = self.store.master[:1]
        outs = _ModelFn.apply(self, batch, dummy.detach().requires_grad_(True))
        tpn, tnn, an = outs[:3]
        self.last_alignment_scores = outs[3] if self.use_word_alignment else None
        return tpn, tnn, an

    # the sub-steps of the reference API (compute_pos_neg_embeddings' building blocks).  Each is
    # differentiable: one autograd node whose backward runs the engine's HIP backward for that
    # block and accumulates parameter gradients into the flat buffer (.grad views), so code
    # written against the reference's methods (ref :508-563) trains unmodified.  Under no_grad
    # they run forward-only without saved activations.
    def encode_text(self, input_ids, attention_mask=None):
        """ref:567-585: (projection [B,P], last_hidden_state [B,L,H])."""
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        ids, mask = input_ids.contiguous(), attention_mask.contiguous()
        if not torch.is_grad_enabled():
            return self._encode_nograd("text", ids, mask)
        return _EncodeFn.apply(self, "text", ids, mask, self.store.master[:1].detach().requires_grad_(True))

    def encode_audio(self, input_values, attention_mask=None):
        """ref:587-641: (projection [B,P], last_hidden_state [B,T,H]).  input_values: w2v-bert
        features [B, T, 160], or raw samples [B, N] for a wav2vec2 audio encoder (whose
        attention_mask may stay None, like wav2vec2-base's processor output)."""
        B, T = input_values.shape[:2]
        if attention_mask is None and not self.engine.raw_audio:
            attention_mask = torch.ones(B, T, dtype=torch.int64, device=input_values.device)
        x, mask = input_values.contiguous(), None if attention_mask is None else attention_mask.contiguous()
        if not torch.is_grad_enabled():
            return self._encode_nograd("audio", x, mask)
        return _EncodeFn.apply(self, "audio", x, mask, self.store.master[:1].detach().requires_grad_(True))

    def apply_cross_modal_attention(self, text_projected, text_hidden, text_mask, audio_projected, audio_hidden,
                                    audio_mask):
        """ref:643-682: (text_fused [B,P], audio_fused [B,P]); identity without use_cross_modal."""
        if not self.use_cross_modal:
            return text_projected, audio_projected
        self.store.sync_shadow()
        if not torch.is_grad_enabled():
            tf, af, _ = self.engine.cross_forward(text_projected, text_hidden, text_mask, audio_projected, audio_hidden,
                                                  audio_mask, self.training, _call_seed(self.training))
            return tf, af
        return _CrossFn.apply(self, text_projected, text_hidden, text_mask, audio_projected, audio_hidden, audio_mask,
                              self.store.master[:1].detach().requires_grad_(True))

    def _encode_nograd(self, kind, x, mask):
        self.store.sync_shadow()
        e = self.engine
        ctx = {}
        if kind == "text":
            B, L = x.shape
            h, hb = e.text_forward(x, mask, self.training, _call_seed(self.training), ctx, save=False)
            m32, pool, proj = ctx["t_mask32"], "text_pooling", "text_projection"
        else:
            h, hb = e.audio_forward(x, mask, self.training, _call_seed(self.training), ctx, save=False)
            B, L = ctx["a_b"], ctx["a_T"]
            m32, pool, proj = ctx["a_mask32"], "audio_pooling", "audio_projection"
        pooled = e._pool_fwd(pool, h, hb, m32, B, L, {}, hs=ctx.get("a_hs"))
        out = e._proj_fwd(proj, pooled, B, self.training, _call_seed(self.training), {})
        return out, h.view(B, L, -1)


def _call_seed(train: bool) -> int:
    """Dropout seed of one API call (counter-based dropout, recomputed in backward)."""
    return int(torch.randint(0, 2**62, (1,)).item()) if train else 0


class _EncodeFn(torch.autograd.Function):
    """encode_text / encode_audio as one autograd node: encoder -> pooling -> projection forward
    on the engine (activations saved), backward = projection, pooling and encoder backward."""

    @staticmethod
    def forward(fctx, model, kind, x, mask, dummy):
        model.store.sync_shadow()
        e = model.engine
        ctx = {}
        train = model.training
        seed = _call_seed(train)
        if kind == "text":
            B, L = x.shape
            h, hb = e.text_forward(x, mask, train, seed, ctx, save=True)
            m32, pool, proj = ctx["t_mask32"], "text_pooling", "text_projection"
        else:
            h, hb = e.audio_forward(x, mask, train, seed, ctx, save=True)
            B, L = ctx["a_b"], ctx["a_T"]
            m32, pool, proj = ctx["a_mask32"], "audio_pooling", "audio_projection"
        sv_pool, sv_proj = {}, {}
        pooled = e._pool_fwd(pool, h, hb, m32, B, L, sv_pool, hs=ctx.get("a_hs"))
        out = e._proj_fwd(proj, pooled, B, train, _site(seed), sv_proj)
        fctx.model, fctx.kind, fctx.ctx = model, kind, ctx
        fctx.saved = (sv_pool, sv_proj, B, L, h.shape[-1], pool, proj)
        return out, h.view(B, L, -1)

    @staticmethod
    def backward(fctx, d_out, d_hidden):
        model, e = fctx.model, fctx.model.engine
        sv_pool, sv_proj, B, L, H, pool, proj = fctx.saved
        model.store.attach_grads()
        if d_hidden is not None:
            dh = d_hidden.reshape(B * L, H).float().contiguous().clone()
        else:
            dh = torch.zeros(B * L, H, device=model.store.device)
        if d_out is not None:
            dpooled = torch.zeros(B, H, device=model.store.device)
            e._proj_bwd(proj, sv_proj, d_out.float().contiguous(), dpooled)
            e._pool_bwd(pool, sv_pool, dpooled, dh, B, L)
        if fctx.kind == "text":
            e.text_backward(dh, fctx.ctx)
        else:
            e.audio_backward(dh, fctx.ctx)
        fctx.ctx = fctx.saved = None
        return None, None, None, None, None


class _CrossFn(torch.autograd.Function):
    """apply_cross_modal_attention as one autograd node (engine.cross_forward / cross_backward)."""

    @staticmethod
    def forward(fctx, model, tproj, th, tmask, aproj, ah, amask, dummy):
        tf, af, sv = model.engine.cross_forward(tproj, th, tmask, aproj, ah, amask, model.training,
                                                _call_seed(model.training))
        fctx.model, fctx.sv = model, sv
        fctx.shapes = (th.shape, ah.shape)
        return tf, af

    @staticmethod
    def backward(fctx, d_tf, d_af):
        model = fctx.model
        sv = fctx.sv
        b = sv["b"]
        P = model.projection_dim
        z = lambda: torch.zeros(b, P, device=model.store.device)  # noqa: E731
        model.store.attach_grads()
        d_tproj, dth, d_aproj, dah = model.engine.cross_backward(sv, d_tf if d_tf is not None else z(),
                                                                 d_af if d_af is not None else z())
        fctx.sv = None
        ts, as_ = fctx.shapes
        return None, d_tproj, dth.view(ts), None, d_aproj, dah.view(as_), None, None


def _site(seed: int) -> int:
    return (seed * 0x9E3779B97F4A7C15 + 1) & ((1 << 62) - 1)


def _l2_normalise(tf_p, tf_n, af):
    """F.normalize(dim=-1) of the three embeddings (ref:561-563) -> ((tpn, tnn, an), norms)."""
    outs = tuple(torch.empty_like(t) for t in (tf_p, tf_n, af))
    norms = [torch.empty(t.shape[0], device=t.device) for t in (tf_p, tf_n, af)]
    for x, y, nrm in zip((tf_p, tf_n, af), outs, norms):
        ops.l2norm_fwd(x.contiguous(), y, nrm)
    return outs, norms


class _ModelFn(torch.autograd.Function):
    """The whole model forward as one autograd node (backward = engine.backward)."""

    @staticmethod
    def forward(fctx, model, batch, dummy):
        tf_p, tf_n, af, align, ctx = model.engine.forward(batch, model.training)
        (tpn, tnn, an), norms = _l2_normalise(tf_p, tf_n, af)
        fctx.model, fctx.ctx = model, ctx
        fctx.saved = (tpn, tnn, an, norms)
        outs = (tpn, tnn, an)
        if align is not None:
            outs = outs + (align,)
        else:
            outs = outs + (torch.zeros(0, device=tpn.device),)
        return outs

    @staticmethod
    def backward(fctx, d_tpn, d_tnn, d_an, d_align):
        model = fctx.model
        tpn, tnn, an, norms = fctx.saved
        grads = []
        for y, nrm, dy in zip((tpn, tnn, an), norms, (d_tpn, d_tnn, d_an)):
            if dy is None:
                dy = torch.zeros_like(y)
            dx = torch.empty_like(y)
            ops.l2norm_bwd(y, nrm, dy.contiguous(), dx)
            grads.append(dx)
        model.store.attach_grads()
        if d_align is not None and d_align.numel() == 0:
            d_align = None
        model.engine.backward(fctx.ctx, grads[0], grads[1], grads[2],
                              None if d_align is None else d_align.contiguous())
        fctx.ctx = None
        return None, None, None


class AlignmentAwareInfoNCE(nn.Module):
    """ref:702-742 — 2-way CE over [s_pos, s_neg]/τ, alignment weighting, corrupt penalty."""

    def __init__(self, temperature=0.1, alignment_weight=0.3, corrupt_gamma=0.35):
        super().__init__()
        self.temperature = temperature
        self.alignment_weight = alignment_weight
        self.corrupt_gamma = corrupt_gamma

    def forward(self, s_pos, s_neg, alignment_scores=None):
        """The ste::pair_loss custom op (torch_ops.py): pair_loss_fwd / pair_loss_bwd kernels."""
        return torch.ops.ste.pair_loss(s_pos, s_neg, alignment_scores, float(self.temperature),
                                       float(self.alignment_weight), float(self.corrupt_gamma))
