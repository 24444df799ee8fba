"""Parameter containers with the reference's exact module tree (state_dict keys).

These nn.Modules only HOLD parameters — no forward math runs through them.  The
math is the HIP schedule in engine.py.  Keeping the reference's attribute names
means checkpoints interchange with the reference (`model.state_dict()` keys,
ref:training/trainer_unfreeze.py:1620 and inference.py strict loads) and the
reference's freezing / optimizer-grouping code paths (which walk
`text_encoder.encoder.layer[i]`, `audio_encoder.encoder.layers[i]`,
`audio_encoder.feature_projection`, names containing 'text_encoder' /
'audio_encoder') keep working unchanged.

Trees:
  text_encoder  = XLMRobertaModel  (tf:models/xlm_roberta/modeling_xlm_roberta.py:56-121,186-463,546-558)
  audio_encoder = Wav2Vec2BertModel (tf:models/wav2vec2_bert/modeling_wav2vec2_bert.py:119-548,921-935)
  heads         = ref:training/trainer_unfreeze.py:66-310, 436-491
"""
from __future__ import annotations

from dataclasses import dataclass, field
from types import SimpleNamespace

from torch import nn


@dataclass
class AudioConfig:
    """w2v-bert-2.0 (transformers Wav2Vec2BertConfig defaults, configuration_wav2vec2_bert.py:139-185)."""
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    feature_projection_input_dim: int = 160
    left_max_position_embeddings: int = 64
    right_max_position_embeddings: int = 8
    conv_depthwise_kernel_size: int = 31
    layer_norm_eps: float = 1e-5
    layerdrop: float = 0.1
    conformer_conv_dropout: float = 0.1
    mask_time_prob: float = 0.05
    mask_time_length: int = 10
    mask_time_min_masks: int = 2


@dataclass
class TextConfig:
    """XLM-R base (paraphrase-multilingual-mpnet-base-v2's encoder)."""
    vocab_size: int = 250002
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 514
    type_vocab_size: int = 1
    layer_norm_eps: float = 1e-5
    pad_token_id: int = 1
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1


# ------------------------------------------------------------------- text (XLM-R)
class _SelfAttn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.query, self.key, self.value = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)


class _Out(nn.Module):
    def __init__(self, din, dout, eps):
        super().__init__()
        self.dense = nn.Linear(din, dout)
        self.LayerNorm = nn.LayerNorm(dout, eps=eps)


class _Attention(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.self = _SelfAttn(d)
        self.output = _Out(d, d, eps)


class _Intermediate(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.dense = nn.Linear(d, f)


class XLMRLayer(nn.Module):
    def __init__(self, c: TextConfig):
        super().__init__()
        self.attention = _Attention(c.hidden_size, c.layer_norm_eps)
        self.intermediate = _Intermediate(c.hidden_size, c.intermediate_size)
        self.output = _Out(c.intermediate_size, c.hidden_size, c.layer_norm_eps)


class _Embeddings(nn.Module):
    def __init__(self, c: TextConfig):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden_size, padding_idx=c.pad_token_id)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size,
                                                padding_idx=c.pad_token_id)


class _Encoder(nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.layer = nn.ModuleList(layers)


class _Pooler(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.dense = nn.Linear(d, d)


class TextEncoder(nn.Module):
    def __init__(self, c: TextConfig):
        super().__init__()
        self.config = c
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder([XLMRLayer(c) for _ in range(c.num_hidden_layers)])
        self.pooler = _Pooler(c.hidden_size)


# ----------------------------------------------------------------- audio (w2v-bert)
class _FeatProj(nn.Module):
    def __init__(self, c: AudioConfig):
        super().__init__()
        self.layer_norm = nn.LayerNorm(c.feature_projection_input_dim, eps=c.layer_norm_eps)
        self.projection = nn.Linear(c.feature_projection_input_dim, c.hidden_size)


class _FFN(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.intermediate_dense = nn.Linear(d, f)
        self.output_dense = nn.Linear(f, d)


class _ConformerAttn(nn.Module):
    def __init__(self, c: AudioConfig):
        super().__init__()
        d = c.hidden_size
        self.linear_q, self.linear_k, self.linear_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.linear_out = nn.Linear(d, d)
        n = c.left_max_position_embeddings + c.right_max_position_embeddings + 1
        self.distance_embedding = nn.Embedding(n, d // c.num_attention_heads)


class _ConvModule(nn.Module):
    def __init__(self, c: AudioConfig):
        super().__init__()
        d, k = c.hidden_size, c.conv_depthwise_kernel_size
        self.layer_norm = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.pointwise_conv1 = nn.Conv1d(d, 2 * d, 1, bias=False)
        self.depthwise_conv = nn.Conv1d(d, d, k, groups=d, bias=False)
        self.depthwise_layer_norm = nn.LayerNorm(d, eps=c.layer_norm_eps)
        self.pointwise_conv2 = nn.Conv1d(d, d, 1, bias=False)


class ConformerLayer(nn.Module):
    def __init__(self, c: AudioConfig):
        super().__init__()
        d, eps = c.hidden_size, c.layer_norm_eps
        self.ffn1_layer_norm = nn.LayerNorm(d, eps=eps)
        self.ffn1 = _FFN(d, c.intermediate_size)
        self.self_attn_layer_norm = nn.LayerNorm(d, eps=eps)
        self.self_attn = _ConformerAttn(c)
        self.conv_module = _ConvModule(c)
        self.ffn2_layer_norm = nn.LayerNorm(d, eps=eps)
        self.ffn2 = _FFN(d, c.intermediate_size)
        self.final_layer_norm = nn.LayerNorm(d, eps=eps)


class _ConformerEncoder(nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.layers = nn.ModuleList(layers)


class AudioEncoder(nn.Module):
    def __init__(self, c: AudioConfig):
        super().__init__()
        self.config = c
        if c.mask_time_prob > 0:
            self.masked_spec_embed = nn.Parameter(nn.init.uniform_(nn.Parameter(_empty(c.hidden_size))))
        self.feature_projection = _FeatProj(c)
        self.encoder = _ConformerEncoder([ConformerLayer(c) for _ in range(c.num_hidden_layers)])


def _empty(*shape):
    import torch
    return torch.empty(*shape)


# --------------------------------------------------------- audio (wav2vec2, raw waveform)
@dataclass
class W2V2Config:
    """wav2vec2-base (transformers Wav2Vec2Config defaults, configuration_wav2vec2.py): the
    raw-waveform encoder of SURVEY §8f rank 4.  Implemented: feat_extract_norm="group",
    conv_bias=False, do_stable_layer_norm=False (post-LN layers), GELU, no adapter."""
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    conv_dim: tuple = (512, 512, 512, 512, 512, 512, 512)
    conv_kernel: tuple = (10, 3, 3, 3, 3, 2, 2)
    conv_stride: tuple = (5, 2, 2, 2, 2, 2, 2)
    num_conv_pos_embeddings: int = 128
    num_conv_pos_embedding_groups: int = 16
    layer_norm_eps: float = 1e-5
    hidden_dropout: float = 0.1
    activation_dropout: float = 0.1
    attention_dropout: float = 0.1
    feat_proj_dropout: float = 0.0
    layerdrop: float = 0.1
    mask_time_prob: float = 0.05
    mask_time_length: int = 10
    mask_time_min_masks: int = 2
    feat_extract_norm: str = "group"
    conv_bias: bool = False
    do_stable_layer_norm: bool = False

    def __post_init__(self):
        if self.feat_extract_norm != "group" or self.conv_bias or self.do_stable_layer_norm:
            raise NotImplementedError("wav2vec2: only the base architecture (feat_extract_norm='group', "
                                      "conv_bias=False, post-LN layers) is implemented")
        self.conv_dim, self.conv_kernel, self.conv_stride = (tuple(self.conv_dim), tuple(self.conv_kernel),
                                                             tuple(self.conv_stride))

    def frames(self, n_samples: int) -> list:
        """Sequence length after each conv layer: [N, T0, T1, ..., T_last]."""
        out = [n_samples]
        for k, s in zip(self.conv_kernel, self.conv_stride):
            out.append((out[-1] - k) // s + 1)
        return out


class _W2VConv(nn.Module):
    def __init__(self, cin, cout, k, s, group_norm):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, k, stride=s, bias=False)
        if group_norm:
            self.layer_norm = nn.GroupNorm(cout, cout, affine=True)


class _W2VFeatureEncoder(nn.Module):
    def __init__(self, c: W2V2Config):
        super().__init__()
        dims = (1,) + c.conv_dim
        self.conv_layers = nn.ModuleList([_W2VConv(dims[i], dims[i + 1], c.conv_kernel[i], c.conv_stride[i], i == 0)
                                          for i in range(len(c.conv_dim))])


class _W2VFeatProj(nn.Module):
    def __init__(self, c: W2V2Config):
        super().__init__()
        self.layer_norm = nn.LayerNorm(c.conv_dim[-1], eps=c.layer_norm_eps)
        self.projection = nn.Linear(c.conv_dim[-1], c.hidden_size)


class _WeightNormParams(nn.Module):
    """nn.utils.parametrizations.weight_norm's parameter holder: state_dict keys
    ...conv.parametrizations.weight.original0 (g [1,1,K]) / original1 (v [D, D/G, K])."""

    def __init__(self, d, cg, k):
        super().__init__()
        import torch
        self.original0 = nn.Parameter(torch.empty(1, 1, k))
        self.original1 = nn.Parameter(torch.empty(d, cg, k))


class _PosConv(nn.Module):
    def __init__(self, c: W2V2Config):
        super().__init__()
        import torch
        d, g, k = c.hidden_size, c.num_conv_pos_embedding_groups, c.num_conv_pos_embeddings
        self.bias = nn.Parameter(torch.empty(d))
        self.parametrizations = nn.Module()
        self.parametrizations.weight = _WeightNormParams(d, d // g, k)


class _PosConvEmbed(nn.Module):
    def __init__(self, c: W2V2Config):
        super().__init__()
        self.conv = _PosConv(c)


class _W2VAttn(nn.Module):
    def __init__(self, d):
        super().__init__()
        # transformers' construction order (k, v, q, out); the ParamStore lays q|k|v out adjacently
        self.k_proj, self.v_proj, self.q_proj = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)


class _W2VFeedForward(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.intermediate_dense = nn.Linear(d, f)
        self.output_dense = nn.Linear(f, d)


class W2V2Layer(nn.Module):
    """Wav2Vec2EncoderLayer (tf:models/wav2vec2/modeling_wav2vec2.py:575-608), post-LN."""

    def __init__(self, c: W2V2Config):
        super().__init__()
        d, eps = c.hidden_size, c.layer_norm_eps
        self.attention = _W2VAttn(d)
        self.layer_norm = nn.LayerNorm(d, eps=eps)
        self.feed_forward = _W2VFeedForward(d, c.intermediate_size)
        self.final_layer_norm = nn.LayerNorm(d, eps=eps)


class _W2VEncoder(nn.Module):
    def __init__(self, c: W2V2Config):
        super().__init__()
        self.pos_conv_embed = _PosConvEmbed(c)
        self.layer_norm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.layers = nn.ModuleList([W2V2Layer(c) for _ in range(c.num_hidden_layers)])


class W2V2AudioEncoder(nn.Module):
    """Wav2Vec2Model's parameter tree (tf:…/modeling_wav2vec2.py:1244-1263): state_dict keys
    match transformers' (feature_extractor.conv_layers.*, feature_projection.*,
    encoder.pos_conv_embed.conv.parametrizations.weight.original0/1, encoder.layers.*)."""

    def __init__(self, c: W2V2Config):
        super().__init__()
        self.config = c
        self.feature_extractor = _W2VFeatureEncoder(c)
        self.feature_projection = _W2VFeatProj(c)
        if c.mask_time_prob > 0:
            self.masked_spec_embed = nn.Parameter(_empty(c.hidden_size))
        self.encoder = _W2VEncoder(c)


# ------------------------------------------------------------------------- heads
class EnhancedProjection(nn.Module):
    """ref:66-99 (Linear -> GELU -> Dropout -> Linear -> LayerNorm)."""

    def __init__(self, input_dim, projection_dim, hidden_dim=None, dropout=0.1):
        super().__init__()
        hidden_dim = hidden_dim or 2 * projection_dim
        self.dropout_p = dropout
        self.projection = nn.Sequential(nn.Linear(input_dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                        nn.Linear(hidden_dim, projection_dim), nn.LayerNorm(projection_dim))


class CrossModalAttention(nn.Module):
    """ref:102-168."""

    def __init__(self, dim, num_heads=8, dropout=0.1):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.dropout_p = dropout
        self.query, self.key, self.value = nn.Linear(dim, dim), nn.Linear(dim, dim), nn.Linear(dim, dim)
        self.out_proj = nn.Linear(dim, dim)
        for m in (self.query, self.key, self.value, self.out_proj):
            nn.init.xavier_uniform_(m.weight)


class AttentivePooling(nn.Module):
    """ref:171-211."""

    def __init__(self, hidden_size):
        super().__init__()
        self.attention = nn.Sequential(nn.Linear(hidden_size, hidden_size // 2), nn.Tanh(),
                                       nn.Linear(hidden_size // 2, 1))


class WordLevelAlignmentModule(nn.Module):
    """ref:214-310."""

    def __init__(self, text_hidden_dim, audio_hidden_dim, alignment_dim, num_heads=4, dropout=0.1):
        super().__init__()
        self.num_heads = num_heads
        self.dropout_p = dropout
        self.text_projection = nn.Linear(text_hidden_dim, alignment_dim)
        self.audio_projection = nn.Linear(audio_hidden_dim, alignment_dim)
        self.alignment_attention = nn.MultiheadAttention(alignment_dim, num_heads, dropout=dropout, batch_first=True)
        self.output_projection = nn.Linear(alignment_dim, alignment_dim)
        self.layer_norm = nn.LayerNorm(alignment_dim)
        self.alignment_confidence = nn.Sequential(nn.Linear(alignment_dim, alignment_dim // 2), nn.ReLU(),
                                                  nn.Linear(alignment_dim // 2, 1))


def config_namespace(**kw):
    return SimpleNamespace(**kw)
