"""ORACLE — test infrastructure, NOT product code.

CPU fp32 restatement (plain torch ops, autograd for gradients) of the reference's
training-step math.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / the timed CPU
baseline — never as part of the product path.

Pinned against the reference itself: tests/golden/make_golden.py runs the real
/root/reference/training/trainer_unfreeze.py model (with transformers 5.15.0,
in this container) and commits its outputs; tests/test_oracle_golden.py checks
this restatement against them.

Functional form: every function takes a flat `params` dict whose keys are the
reference's state_dict keys (EnhancedAudioTextModel module tree), so weights
interchange with the reference and with the GPU model.

Citations:
  ref: = /root/reference/training/trainer_unfreeze.py
  w2v: = transformers/models/wav2vec2_bert/modeling_wav2vec2_bert.py
  xlm: = transformers/models/xlm_roberta/modeling_xlm_roberta.py
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

FINFO_MIN = torch.finfo(torch.float32).min


@dataclass
class AudioCfg:  # w2v: configuration_wav2vec2_bert.py:139-185 (w2v-bert-2.0 defaults)
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    inter: int = 4096
    feat_in: int = 160
    left: int = 64
    right: int = 8
    conv_k: int = 31
    eps: float = 1e-5


@dataclass
class TextCfg:  # XLM-R base as shipped by paraphrase-multilingual-mpnet-base-v2
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    inter: int = 3072
    vocab: int = 250002
    max_pos: int = 514
    pad_id: int = 1
    eps: float = 1e-5


@dataclass
class ModelCfg:  # ref:324-338 constructor arguments
    audio: AudioCfg = field(default_factory=AudioCfg)
    text: TextCfg = field(default_factory=TextCfg)
    projection_dim: int = 768
    use_cross_modal: bool = True
    use_attentive_pooling: bool = True
    use_word_alignment: bool = False
    text_layers_to_unfreeze: int = 3
    audio_layers_to_unfreeze: int = 3
    xattn_heads: int = 8       # ref:102 CrossModalAttention(num_heads=8)
    align_heads: int = 4       # ref:218 WordLevelAlignmentModule(num_heads=4)


# ------------------------------------------------------------------ helpers
def _lin(p, name, x):
    w = p[name + ".weight"]
    b = p.get(name + ".bias")
    return F.linear(x, w, b)


def _ln(p, name, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


# ------------------------------------------------------------ audio encoder
def conformer_self_attn(p, pre, h, add_mask, cfg: AudioCfg):
    """w2v:229-327, relative_key branch: scores = (QKᵀ + Q·E[clamp(r-l)])/sqrt(d) + mask."""
    B, T, D = h.shape
    H, d = cfg.heads, D // cfg.heads
    q = _lin(p, pre + "linear_q", h).view(B, T, H, d).transpose(1, 2)
    k = _lin(p, pre + "linear_k", h).view(B, T, H, d).transpose(1, 2)
    v = _lin(p, pre + "linear_v", h).view(B, T, H, d).transpose(1, 2)
    scores = q @ k.transpose(-2, -1) / math.sqrt(d)
    pos = torch.arange(T)
    dist = (pos.view(1, -1) - pos.view(-1, 1)).clamp(-cfg.left, cfg.right) + cfg.left  # [l, r]
    E = p[pre + "distance_embedding.weight"]                                          # [left+right+1, d]
    qe = q @ E.t()                                                                    # [B,H,T,nrel]
    rel = torch.gather(qe, 3, dist.view(1, 1, T, T).expand(B, H, T, T))              # == einsum bhld,lrd
    scores = scores + rel / math.sqrt(d)
    if add_mask is not None:
        scores = scores + add_mask
    probs = torch.softmax(scores, dim=-1)
    o = (probs @ v).transpose(1, 2).reshape(B, T, D)
    return _lin(p, pre + "linear_out", o)


def conformer_conv(p, pre, h, mask, cfg: AudioCfg):
    """w2v:157-226: LN -> masked_fill -> pw1 -> GLU -> causal depthwise -> LN -> swish -> pw2."""
    x = _ln(p, pre + "layer_norm", h, cfg.eps)
    if mask is not None:
        x = x.masked_fill(~mask.bool().unsqueeze(-1), 0.0)
    x = x.transpose(1, 2)
    x = F.conv1d(x, p[pre + "pointwise_conv1.weight"])
    x = F.glu(x, dim=1)
    x = F.pad(x, (cfg.conv_k - 1, 0))
    x = F.conv1d(x, p[pre + "depthwise_conv.weight"], groups=x.shape[1])
    x = _ln(p, pre + "depthwise_layer_norm", x.transpose(1, 2), cfg.eps).transpose(1, 2)
    x = F.silu(x)
    x = F.conv1d(x, p[pre + "pointwise_conv2.weight"])
    return x.transpose(1, 2)


def conformer_ffn(p, pre, h):
    """w2v:134-154 (swish, dropouts are 0 in the w2v-bert config)."""
    return _lin(p, pre + "output_dense", F.silu(_lin(p, pre + "intermediate_dense", h)))


def audio_encoder(p, feats, mask, cfg: AudioCfg, prefix="audio_encoder.", spec_mask=None):
    """w2v:991-1042 (Wav2Vec2BertModel.forward) + encoder w2v:480-548.  spec_mask (bool [B,T],
    training mode): SpecAugment rows replaced by masked_spec_embed (w2v:944-988) before the
    encoder zeroes the padded frames."""
    x = _ln(p, prefix + "feature_projection.layer_norm", feats, cfg.eps)
    h = _lin(p, prefix + "feature_projection.projection", x)
    if spec_mask is not None:
        h = torch.where(spec_mask.unsqueeze(-1), p[prefix + "masked_spec_embed"].expand_as(h), h)
    add_mask = None
    if mask is not None:
        h = h.masked_fill(~mask.bool().unsqueeze(-1), 0.0)
        add_mask = (1.0 - mask[:, None, None, :].to(h.dtype)) * FINFO_MIN
    for i in range(cfg.layers):
        pre = f"{prefix}encoder.layers.{i}."
        r = h
        h = conformer_ffn(p, pre + "ffn1.", _ln(p, pre + "ffn1_layer_norm", h, cfg.eps)) * 0.5 + r
        r = h
        h = conformer_self_attn(p, pre + "self_attn.", _ln(p, pre + "self_attn_layer_norm", h, cfg.eps), add_mask,
                                cfg) + r
        r = h
        h = r + conformer_conv(p, pre + "conv_module.", h, mask, cfg)
        r = h
        h = conformer_ffn(p, pre + "ffn2.", _ln(p, pre + "ffn2_layer_norm", h, cfg.eps)) * 0.5 + r
        h = _ln(p, pre + "final_layer_norm", h, cfg.eps)
    return h


# ------------------------------------------------------------- text encoder
def text_encoder(p, ids, mask, cfg: TextCfg, prefix="text_encoder."):
    """xlm:75-121 embeddings (+ position ids xlm:142-155) and 12 post-LN layers xlm:186-463 (eval)."""
    B, L = ids.shape
    nz = (ids != cfg.pad_id).int()
    pos_ids = (torch.cumsum(nz, dim=1) * nz).long() + cfg.pad_id
    # nn.Embedding(padding_idx=pad): the pad row receives no gradient (word ids == pad, and the
    # position ids of pad tokens == pad, xlm:142-155)
    e = (F.embedding(ids, p[prefix + "embeddings.word_embeddings.weight"], padding_idx=cfg.pad_id)
         + p[prefix + "embeddings.token_type_embeddings.weight"][0]
         + F.embedding(pos_ids, p[prefix + "embeddings.position_embeddings.weight"], padding_idx=cfg.pad_id))
    x = _ln(p, prefix + "embeddings.LayerNorm", e, cfg.eps)
    add_mask = None
    if mask is not None:
        add_mask = (1.0 - mask[:, None, None, :].to(x.dtype)) * FINFO_MIN
    H, d = cfg.heads, cfg.hidden // cfg.heads
    for i in range(cfg.layers):
        pre = f"{prefix}encoder.layer.{i}."
        q = _lin(p, pre + "attention.self.query", x).view(B, L, H, d).transpose(1, 2)
        k = _lin(p, pre + "attention.self.key", x).view(B, L, H, d).transpose(1, 2)
        v = _lin(p, pre + "attention.self.value", x).view(B, L, H, d).transpose(1, 2)
        s = q @ k.transpose(-2, -1) / math.sqrt(d)
        if add_mask is not None:
            s = s + add_mask
        pr = torch.softmax(s, -1)
        if mask is not None:
            # the reference's XLM-R attention is SDPA (transformers 5.15 in this container), whose
            # boolean mask gives a query with every key masked zero weights (torch's safe softmax),
            # not the uniform weights of an additive finfo.min mask (pinned by model_golden_masked)
            pr = pr * (mask.sum(1) > 0).to(pr.dtype)[:, None, None, None]
        o = (pr @ v).transpose(1, 2).reshape(B, L, cfg.hidden)
        x = _ln(p, pre + "attention.output.LayerNorm", _lin(p, pre + "attention.output.dense", o) + x, cfg.eps)
        inter = F.gelu(_lin(p, pre + "intermediate.dense", x))
        x = _ln(p, pre + "output.LayerNorm", _lin(p, pre + "output.dense", inter) + x, cfg.eps)
    return x


# -------------------------------------------------------------------- heads
def enhanced_projection(p, pre, x):
    """ref:66-99: Linear -> GELU -> Dropout -> Linear -> LayerNorm."""
    h = F.gelu(_lin(p, pre + "projection.0", x))
    return _ln(p, pre + "projection.4", _lin(p, pre + "projection.3", h))


def attentive_pooling(p, pre, h, mask):
    """ref:171-211."""
    s = _lin(p, pre + "attention.2", torch.tanh(_lin(p, pre + "attention.0", h))).squeeze(-1)
    if mask is not None:
        s = s.masked_fill(mask == 0, -1e9)
    w = torch.softmax(s, dim=1)
    return torch.bmm(w.unsqueeze(1), h).squeeze(1)


def cross_modal_attention(p, pre, x, ctx, mask, heads):
    """ref:125-168 (x: [B,1,P] single query)."""
    B = x.shape[0]
    P = x.shape[-1]
    d = P // heads
    q = _lin(p, pre + "query", x).view(B, -1, heads, d).transpose(1, 2)
    k = _lin(p, pre + "key", ctx).view(B, -1, heads, d).transpose(1, 2)
    v = _lin(p, pre + "value", ctx).view(B, -1, heads, d).transpose(1, 2)
    a = (q @ k.transpose(-2, -1)) * d ** -0.5
    if mask is not None:
        a = a.masked_fill(mask.unsqueeze(1).unsqueeze(2) == 0, -1e9)
    a = torch.softmax(a, dim=-1)
    o = (a @ v).transpose(1, 2).contiguous().view(B, -1, heads * d)
    return _lin(p, pre + "out_proj", o)


def word_level_alignment(p, pre, text_h, audio_h, text_mask, audio_mask, heads):
    """ref:250-310 (nn.MultiheadAttention batch_first, eval)."""
    tp = _lin(p, pre + "text_projection", text_h)
    ap = _lin(p, pre + "audio_projection", audio_h)
    B, L, E = tp.shape
    S = ap.shape[1]
    W = p[pre + "alignment_attention.in_proj_weight"]
    bW = p[pre + "alignment_attention.in_proj_bias"]
    q = F.linear(tp, W[:E], bW[:E])
    k = F.linear(ap, W[E:2 * E], bW[E:2 * E])
    v = F.linear(ap, W[2 * E:], bW[2 * E:])
    d = E // heads
    q = q.view(B, L, heads, d).transpose(1, 2)
    k = k.view(B, S, heads, d).transpose(1, 2)
    v = v.view(B, S, heads, d).transpose(1, 2)
    s = (q @ k.transpose(-2, -1)) / math.sqrt(d)
    if audio_mask is not None:
        kpm = (1.0 - audio_mask).bool()
        s = s.masked_fill(kpm[:, None, None, :], float("-inf"))
    w = torch.softmax(s, dim=-1)
    o = (w @ v).transpose(1, 2).reshape(B, L, E)
    o = _lin(p, pre + "alignment_attention.out_proj", o)
    aligned = _ln(p, pre + "layer_norm", text_h + _lin(p, pre + "output_projection", o))
    sc = _lin(p, pre + "alignment_confidence.2", F.relu(_lin(p, pre + "alignment_confidence.0", aligned))).squeeze(-1)
    if text_mask is not None:
        sc = sc * text_mask
    return sc


def encode_text(p, ids, mask, cfg: ModelCfg):
    """ref:567-585."""
    h = text_encoder(p, ids, mask, cfg.text)
    pooled = attentive_pooling(p, "text_pooling.", h, mask) if cfg.use_attentive_pooling else h[:, 0]
    return enhanced_projection(p, "text_projection.", pooled), h


def encode_audio(p, feats, mask, cfg: ModelCfg, spec_mask=None):
    """ref:587-641."""
    h = audio_encoder(p, feats, mask, cfg.audio, spec_mask=spec_mask)
    if cfg.use_attentive_pooling:
        pooled = attentive_pooling(p, "audio_pooling.", h, mask)
    else:
        m = mask.unsqueeze(-1).to(h.dtype)
        pooled = (h * m).sum(1) / m.sum(1).clamp(min=1e-9)
    return enhanced_projection(p, "audio_projection.", pooled), h


def apply_cross_modal(p, tproj, th, tmask, aproj, ah, amask, cfg: ModelCfg):
    """ref:643-682."""
    aseq = _lin(p, "audio_seq_to_projection", ah)
    tseq = _lin(p, "text_seq_to_projection", th)
    t_att = cross_modal_attention(p, "text_to_audio_attention.", tproj.unsqueeze(1), aseq, amask,
                                  cfg.xattn_heads).squeeze(1)
    a_att = cross_modal_attention(p, "audio_to_text_attention.", aproj.unsqueeze(1), tseq, tmask,
                                  cfg.xattn_heads).squeeze(1)
    tf_ = _ln(p, "text_fusion.1", _lin(p, "text_fusion.0", torch.cat([tproj, t_att], 1)))
    af_ = _ln(p, "audio_fusion.1", _lin(p, "audio_fusion.0", torch.cat([aproj, a_att], 1)))
    return tf_, af_


def compute_pos_neg_embeddings(p, batch, cfg: ModelCfg, spec_mask=None):
    """ref:502-565.  Returns (txt_pos_norm, txt_neg_norm, aud_norm, alignment_scores|None).
    spec_mask: the training-mode SpecAugment rows of the audio encoder (None: eval / off)."""
    tp, th = encode_text(p, batch["input_ids_pos"], batch["attention_mask_pos"], cfg)
    tn, thn = encode_text(p, batch["input_ids_neg"], batch["attention_mask_neg"], cfg)
    ap, ah = encode_audio(p, batch["input_values"], batch["attention_mask_audio"], cfg, spec_mask=spec_mask)
    if cfg.use_cross_modal:
        tpf, af = apply_cross_modal(p, tp, th, batch["attention_mask_pos"], ap, ah, batch["attention_mask_audio"], cfg)
        tnf, _ = apply_cross_modal(p, tn, thn, batch["attention_mask_neg"], ap, ah, batch["attention_mask_audio"], cfg)
    else:
        tpf, tnf, af = tp, tn, ap
    align = None
    if cfg.use_word_alignment:
        align = word_level_alignment(p, "word_level_alignment.", th, ah, batch["attention_mask_pos"],
                                     batch["attention_mask_audio"], cfg.align_heads)
    return F.normalize(tpf, p=2, dim=1), F.normalize(tnf, p=2, dim=1), F.normalize(af, p=2, dim=1), align


def alignment_aware_infonce(s_pos, s_neg, align=None, temperature=0.1, alignment_weight=0.5, corrupt_gamma=0.35):
    """ref:702-742."""
    logits = torch.stack([s_pos, s_neg], dim=1) / temperature
    per = F.cross_entropy(logits, torch.zeros(logits.shape[0], dtype=torch.long), reduction="none")
    if align is not None:
        per = per * (1.0 - torch.sigmoid(align.mean(dim=1)) * alignment_weight)
    loss = per.mean()
    if corrupt_gamma > 0:
        loss = loss + corrupt_gamma * F.relu(s_neg).mean()
    return loss


def step_loss(p, batch, cfg: ModelCfg, loss_kw=None):
    """Forward of one train_epoch iteration (ref:1068-1081) -> (loss, s_pos, s_neg, embeddings)."""
    tpn, tnn, an, align = compute_pos_neg_embeddings(p, batch, cfg)
    s_pos = (an * tpn).sum(1)
    s_neg = (an * tnn).sum(1)
    loss = alignment_aware_infonce(s_pos, s_neg, align, **(loss_kw or {}))
    return loss, s_pos, s_neg, (tpn, tnn, an, align)


# ---------------------------------------------------------- freezing rules
def trainable_names(names, cfg: ModelCfg):
    """ref:355-434 partial freezing: returns the set of parameter names with requires_grad=True."""
    out = set()
    nt, na = cfg.text.layers, cfg.audio.layers
    for n in names:
        if n.startswith("text_encoder.encoder.layer."):
            i = int(n.split(".")[3])
            if i >= nt - cfg.text_layers_to_unfreeze:
                out.add(n)
        elif n.startswith("audio_encoder.encoder.layers."):
            i = int(n.split(".")[3])
            if i >= na - cfg.audio_layers_to_unfreeze:
                out.add(n)
        else:
            out.add(n)
    return out


def adamw_step(p, g, m, v, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.01, step=1):
    """torch.optim.AdamW single-tensor update (decoupled decay), restated."""
    p = p * (1 - lr * wd)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def linear_warmup_lr(base_lr, step, warmup, total):
    """transformers get_linear_schedule_with_warmup lr_lambda (ref:1537-1541)."""
    if step < warmup:
        return base_lr * step / max(1, warmup)
    return base_lr * max(0.0, (total - step) / max(1, total - warmup))


# ------------------------------------------------------- module-tree shapes
def param_shapes(cfg: ModelCfg, spec_augment: bool = True):
    """Ordered (state_dict key, shape) of the reference EnhancedAudioTextModel (ref:315-491 +
    XLMRobertaModel / Wav2Vec2BertModel trees).  spec_augment: w2v config has mask_time_prob>0
    (w2v:930-931 creates masked_spec_embed)."""
    t, a, P = cfg.text, cfg.audio, cfg.projection_dim
    out = []
    add = lambda n, *s: out.append((n, tuple(s)))  # noqa: E731
    e = "text_encoder.embeddings."
    add(e + "word_embeddings.weight", t.vocab, t.hidden)
    add(e + "token_type_embeddings.weight", 1, t.hidden)
    add(e + "LayerNorm.weight", t.hidden); add(e + "LayerNorm.bias", t.hidden)
    add(e + "position_embeddings.weight", t.max_pos, t.hidden)
    for i in range(t.layers):
        pre = f"text_encoder.encoder.layer.{i}."
        for n in ("query", "key", "value"):
            add(pre + f"attention.self.{n}.weight", t.hidden, t.hidden); add(pre + f"attention.self.{n}.bias", t.hidden)
        add(pre + "attention.output.dense.weight", t.hidden, t.hidden); add(pre + "attention.output.dense.bias", t.hidden)
        add(pre + "attention.output.LayerNorm.weight", t.hidden); add(pre + "attention.output.LayerNorm.bias", t.hidden)
        add(pre + "intermediate.dense.weight", t.inter, t.hidden); add(pre + "intermediate.dense.bias", t.inter)
        add(pre + "output.dense.weight", t.hidden, t.inter); add(pre + "output.dense.bias", t.hidden)
        add(pre + "output.LayerNorm.weight", t.hidden); add(pre + "output.LayerNorm.bias", t.hidden)
    add("text_encoder.pooler.dense.weight", t.hidden, t.hidden); add("text_encoder.pooler.dense.bias", t.hidden)
    if spec_augment:
        add("audio_encoder.masked_spec_embed", a.hidden)
    f = "audio_encoder.feature_projection."
    add(f + "layer_norm.weight", a.feat_in); add(f + "layer_norm.bias", a.feat_in)
    add(f + "projection.weight", a.hidden, a.feat_in); add(f + "projection.bias", a.hidden)
    dh = a.hidden // a.heads
    for i in range(a.layers):
        pre = f"audio_encoder.encoder.layers.{i}."
        ln = lambda n: (add(pre + n + ".weight", a.hidden), add(pre + n + ".bias", a.hidden))  # noqa: E731
        ln("ffn1_layer_norm")
        add(pre + "ffn1.intermediate_dense.weight", a.inter, a.hidden); add(pre + "ffn1.intermediate_dense.bias", a.inter)
        add(pre + "ffn1.output_dense.weight", a.hidden, a.inter); add(pre + "ffn1.output_dense.bias", a.hidden)
        ln("self_attn_layer_norm")
        for n in ("linear_q", "linear_k", "linear_v", "linear_out"):
            add(pre + f"self_attn.{n}.weight", a.hidden, a.hidden); add(pre + f"self_attn.{n}.bias", a.hidden)
        add(pre + "self_attn.distance_embedding.weight", a.left + a.right + 1, dh)
        ln("conv_module.layer_norm")
        add(pre + "conv_module.pointwise_conv1.weight", 2 * a.hidden, a.hidden, 1)
        add(pre + "conv_module.depthwise_conv.weight", a.hidden, 1, a.conv_k)
        ln("conv_module.depthwise_layer_norm")
        add(pre + "conv_module.pointwise_conv2.weight", a.hidden, a.hidden, 1)
        ln("ffn2_layer_norm")
        add(pre + "ffn2.intermediate_dense.weight", a.inter, a.hidden); add(pre + "ffn2.intermediate_dense.bias", a.inter)
        add(pre + "ffn2.output_dense.weight", a.hidden, a.inter); add(pre + "ffn2.output_dense.bias", a.hidden)
        ln("final_layer_norm")
    for side, H in (("text", t.hidden), ("audio", a.hidden)):
        pre = f"{side}_projection.projection."
        add(pre + "0.weight", 2 * P, H); add(pre + "0.bias", 2 * P)
        add(pre + "3.weight", P, 2 * P); add(pre + "3.bias", P)
        add(pre + "4.weight", P); add(pre + "4.bias", P)
    if cfg.use_cross_modal:
        add("text_seq_to_projection.weight", P, t.hidden); add("text_seq_to_projection.bias", P)
        add("audio_seq_to_projection.weight", P, a.hidden); add("audio_seq_to_projection.bias", P)
        for m in ("text_to_audio_attention", "audio_to_text_attention"):
            for n in ("query", "key", "value", "out_proj"):
                add(f"{m}.{n}.weight", P, P); add(f"{m}.{n}.bias", P)
        for m in ("text_fusion", "audio_fusion"):
            add(f"{m}.0.weight", P, 2 * P); add(f"{m}.0.bias", P)
            add(f"{m}.1.weight", P); add(f"{m}.1.bias", P)
    if cfg.use_attentive_pooling:
        for side, H in (("text", t.hidden), ("audio", a.hidden)):
            pre = f"{side}_pooling.attention."
            add(pre + "0.weight", H // 2, H); add(pre + "0.bias", H // 2)
            add(pre + "2.weight", 1, H // 2); add(pre + "2.bias", 1)
    if cfg.use_word_alignment:
        w = "word_level_alignment."
        add(w + "text_projection.weight", P, t.hidden); add(w + "text_projection.bias", P)
        add(w + "audio_projection.weight", P, a.hidden); add(w + "audio_projection.bias", P)
        add(w + "alignment_attention.in_proj_weight", 3 * P, P); add(w + "alignment_attention.in_proj_bias", 3 * P)
        add(w + "alignment_attention.out_proj.weight", P, P); add(w + "alignment_attention.out_proj.bias", P)
        add(w + "output_projection.weight", P, P); add(w + "output_projection.bias", P)
        add(w + "layer_norm.weight", P); add(w + "layer_norm.bias", P)
        add(w + "alignment_confidence.0.weight", P // 2, P); add(w + "alignment_confidence.0.bias", P // 2)
        add(w + "alignment_confidence.2.weight", 1, P // 2); add(w + "alignment_confidence.2.bias", 1)
    return out


def mini_cfg(golden_json: dict) -> ModelCfg:
    m = golden_json["mini"]
    au, tx = m["audio"], m["text"]
    return ModelCfg(
        audio=AudioCfg(hidden=au["hidden_size"], layers=au["num_hidden_layers"], heads=au["num_attention_heads"],
                       inter=au["intermediate_size"], feat_in=au["feature_projection_input_dim"],
                       left=au["left_max_position_embeddings"], right=au["right_max_position_embeddings"],
                       conv_k=au["conv_depthwise_kernel_size"]),
        text=TextCfg(hidden=tx["hidden_size"], layers=tx["num_hidden_layers"], heads=tx["num_attention_heads"],
                     inter=tx["intermediate_size"], vocab=tx["vocab_size"], max_pos=tx["max_position_embeddings"],
                     pad_id=tx["pad_token_id"]),
        projection_dim=m["projection_dim"], use_word_alignment=golden_json["use_word_alignment"],
        use_attentive_pooling=golden_json.get("use_attentive_pooling", True),
        text_layers_to_unfreeze=m["unfreeze"], audio_layers_to_unfreeze=m["unfreeze"])
