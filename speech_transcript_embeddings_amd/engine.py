"""The hot path as an explicit HIP schedule: forward and backward of the whole
contrastive step (two encoders + heads), every op a libste.so kernel.

Reference call stack being replaced (ref = /root/reference/training/trainer_unfreeze.py):
  EnhancedAudioTextModel.compute_pos_neg_embeddings  ref:502-565
    encode_text x2 (pos, neg)                        ref:567-585  -> XLM-R (batched pos+neg here)
    encode_audio                                     ref:587-641  -> Wav2Vec2Bert (Conformer)
    apply_cross_modal_attention x2                   ref:643-682
    word_level_alignment (optional)                  ref:550-558
    F.normalize x3                                   ref:561-563
and the autograd backward of all of it.

Data layout in HBM: activations are row-major [rows, features]; rows = batch*time
(audio) or 2*batch*tokens (text, pos rows then neg rows).  Residual streams and
LayerNorm inputs are fp32; every GEMM operand is bf16 (MFMA), accumulation fp32.
Backward writes parameter gradients straight into the flat gradient buffer of
store.py (beta=1 accumulation), so micro-batch accumulation needs no extra pass.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib, ops
from ._lib import (ACT_GELU, ACT_GELU_BWD, ACT_NONE, ACT_RELU, ACT_RELU_BWD, ACT_SWISH, ACT_SWISH_BWD,
                   ACT_TANH)

BF16, F32 = torch.bfloat16, torch.float32
_GOLD = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


def _site_seed(base: int, site: int) -> int:
    x = (base + (site + 1) * _GOLD) & _M64
    x ^= x >> 31
    return (x * 0xBF58476D1CE4E5B9) & _M64


# parameter names of the post-LN layer (Engine._postln_fwd / _postln_bwd)
XLMR_NAMES = dict(layer="text_encoder.encoder.layer.{i}.", q="attention.self.query", o="attention.output.dense",
                  ln1="attention.output.LayerNorm", fi="intermediate.dense", fo="output.dense", ln2="output.LayerNorm")
W2V2_NAMES = dict(layer="audio_encoder.encoder.layers.{i}.", q="attention.q_proj", o="attention.out_proj",
                  ln1="layer_norm", fi="feed_forward.intermediate_dense", fo="feed_forward.output_dense",
                  ln2="final_layer_norm")


class Ctx(dict):
    """Saved activations of one forward (freed when backward finishes)."""


class Engine:
    def __init__(self, model):
        self.m = model
        self.s = model.store
        self.acfg = model.audio_cfg
        self.tcfg = model.text_cfg
        self._ws = {}
        self._side = None
        # the text encoder (forward and backward) runs on a second HIP stream, concurrently with
        # the audio encoder: its GEMMs are too small to fill 256 CUs (8,192 rows) and overlap the
        # audio side's bandwidth-bound kernels.  STE_TEXT_STREAM=0: one stream (A/B runs).
        self.overlap = os.environ.get("STE_TEXT_STREAM", "1") != "0"
        # layerdrop draws (tf:…wav2vec2_bert…:519-522): the global torch RNG unless a trainer sets a
        # generator (TrainStep broadcasts one seed so every data-parallel rank drops the same layers)
        self.layerdrop_gen = None
        # a Conformer layer's final LN and the next layer's FFN1 LN as one fused pass (forward and
        # backward, ste_layernorm_*_pair); STE_LN_PAIR=0: separate launches (A/B runs)
        self.ln_pair = os.environ.get("STE_LN_PAIR", "1") != "0"

    @property
    def fp8(self):
        """MX-fp8 forward GEMMs in the Conformer layers (model fp8_gemm=True, BASELINE config 5)."""
        return bool(getattr(self.m, "fp8_gemm", False))

    WS_BYTES = 80 << 20   # split-K slabs of the weight-gradient GEMMs (largest: 7 x 3072 x 768 fp32)

    @property
    def ws(self):
        """Split-K workspace of the CURRENT stream (the text and audio backward run concurrently)."""
        key = torch.cuda.current_stream(self.s.device).cuda_stream if self.s.device.type == "cuda" else 0
        w = self._ws.get(key)
        if w is None:
            w = self._ws[key] = torch.empty(self.WS_BYTES // 4, device=self.s.device, dtype=F32)
        return w

    def _side_stream(self):
        if not (self.overlap and self.s.device.type == "cuda"):
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.s.device)
        return self._side

    # ------------------------------------------------------------- helpers
    def _e(self, *shape, dtype=F32):
        return torch.empty(shape, device=self.s.device, dtype=dtype)

    def _z(self, *shape, dtype=F32):
        return torch.zeros(shape, device=self.s.device, dtype=dtype)

    def _dw(self, dy_b, x_b, wname, fused=1):
        """dW[N,K] += dyᵀ·x into the flat gradient buffer (if the weight receives gradients)."""
        g = self.s.fused(wname, fused, "g") if fused > 1 else self.s.g(wname)
        if g is None:
            return
        g2 = g.view(g.shape[0], -1)
        ops.linear_dw(dy_b, x_b, out=g2, beta=1.0, ws=self.ws)

    def _dx(self, dy, wname, fused=1, **kw):
        """dX = dY·W of an encoder Linear on the KC-KC GEMM with the cached k-contiguous Wᵀ
        (ParamStore.wt): 15-20 % faster than reading W k-major through transposing LDS reads,
        and bit-identical to it (same reduction order)."""
        return ops.linear(dy, self.s.wt(wname, fused), **kw)

    def _db(self, x, bname, fused=1):
        g = self.s.fused(bname, fused, "g") if fused > 1 else self.s.g(bname)
        if g is not None:
            ops.colsum(x, g)

    def _ln(self, x, name, eps, **kw):
        return ops.layernorm_fwd(x, self.s.p(name + ".weight"), self.s.p(name + ".bias"), eps, **kw)

    def _ln_bwd(self, dy, x, stats, name, **kw):
        g = self.s.g(name + ".weight")
        return ops.layernorm_bwd(dy, x, stats[0], stats[1], self.s.p(name + ".weight"), beta=self.s.p(name + ".bias"),
                                 dgamma=g, dbeta=self.s.g(name + ".bias"), **kw)

    # ================================================================ audio
    @property
    def raw_audio(self):
        """wav2vec2 raw-waveform encoder (wav2vec2.py) instead of w2v-bert's fbank Conformer."""
        from .modules import W2V2Config
        return isinstance(self.acfg, W2V2Config)

    def audio_forward(self, feats, mask_i64, train, base_seed, ctx, save=True):
        if self.raw_audio:
            from . import wav2vec2
            return wav2vec2.forward(self, feats, mask_i64, train, base_seed, ctx, save)
        c = self.acfg
        b, T, fin = feats.shape
        M = b * T
        D = c.hidden_size
        maskf = self._e(M)
        mask32 = self._e(M, dtype=torch.int32)
        _lib.call("ste_mask_i64_to_f32", mask_i64.data_ptr(), maskf.data_ptr(), mask32.data_ptr(), M,
                  _lib.stream_ptr())
        xin = feats.reshape(M, fin)
        a0 = self._e(M, fin, dtype=BF16)
        st0 = self._ln(xin, "audio_encoder.feature_projection.layer_norm", c.layer_norm_eps, yb=a0)
        x = ops.linear(a0, self.s.w("audio_encoder.feature_projection.projection.weight"),
                       self.s.p("audio_encoder.feature_projection.projection.bias"), row_scale=maskf)
        spec = None
        if train and getattr(self.m, "spec_augment", False) and c.mask_time_prob > 0:
            # SpecAugment (w2v:944-988): spans drawn on the host with numpy's global RNG exactly as
            # transformers does (the frame counts cost one host sync, as in the reference)
            from .specaug import compute_mask_indices
            sm = compute_mask_indices((b, T), c.mask_time_prob, c.mask_time_length, mask_i64.sum(-1).tolist(),
                                      c.mask_time_min_masks)
            spec = torch.from_numpy(sm.astype("int32").reshape(-1)).to(self.s.device)
            ops.spec_mask_fwd(x, spec, maskf, self.s.p("audio_encoder.masked_spec_embed"))
        ctx.update(a_b=b, a_T=T, a_maskf=maskf, a_mask32=mask32, a_xin=xin, a_a0=a0, a_st0=st0, a_spec=spec)
        xb = None
        nl = c.num_hidden_layers
        # layerdrop draws (one per layer, in layer order, as transformers does) made up front so
        # each layer knows the next one that runs (its FFN1 LN fuses with this layer's final LN)
        run = [not (train and c.layerdrop > 0 and float(torch.rand([], generator=self.layerdrop_gen)) < c.layerdrop)
               for _ in range(nl)]
        order = [i for i in range(nl) if run[i]]
        layers = [None] * nl
        pre1 = None
        for k, i in enumerate(order):
            last = i == nl - 1
            nxt = order[k + 1] if (self.ln_pair and k + 1 < len(order)) else None
            x, xb, sv, pre1 = self._conformer_fwd(i, x, b, T, maskf, mask32, train, _site_seed(base_seed, 100 + i),
                                                  last, save, pre1=pre1, nxt=nxt)
            layers[i] = sv if save else None
        if xb is None:  # the last layer was dropped (only the last layer writes the bf16 copy)
            xb = ops.cast_bf16(x, self._e(M, D, dtype=BF16))
        ctx["a_layers"] = layers
        return x, xb

    def _conformer_fwd(self, i, x, b, T, maskf, mask32, train, seed, want_bf16, save=True, pre1=None, nxt=None):
        """One Conformer layer.  pre1 = (a1, a1in, stats): this layer's FFN1 LN, already computed
        by the previous layer's fused final-LN pair; nxt = index of the next layer that runs
        (None: none, or no fusion): its FFN1 LN is computed here, fused with this final LN.
        -> (x5, x5 bf16 or None, saved activations, pre1 of layer nxt)."""
        c = self.acfg
        s = self.s
        pre = f"audio_encoder.encoder.layers.{i}."
        M, D, F_ = x.shape[0], c.hidden_size, c.intermediate_size
        H = c.num_attention_heads
        eps = c.layer_norm_eps
        tr = s.trainable_layer(pre + "ffn1_layer_norm.weight")
        sv = {"tr": tr, "seed": seed}
        fp8 = self.fp8

        def lin(xb, wname, bias, count=1, **kw):
            """Forward nn.Linear: bf16 MFMA, or MX-fp8 (fp8_gemm: x block-quantised here unless it
            arrives quantised as an (e4m3, scales) pair, W from ParamStore.wq)."""
            if fp8:
                xq = xb if isinstance(xb, tuple) else ops.mx8_quant(xb)
                return ops.linear_mx8(xq, s.wq(wname, count), bias, **kw)
            return ops.linear(xb, s.fused(wname, count, "w") if count > 1 else s.w(wname), bias, **kw)

        def ffn_in(a, wname, bname, z):
            """FFN intermediate (swish): bf16 output, and under fp8_gemm the MX-fp8 copy the output
            GEMM reads; the bf16 copy is kept only for the trained layers' weight gradients."""
            if not fp8:
                h = lin(a, wname, s.p(bname), act=ACT_SWISH, pre_out=z, out_bf16=True)
                return h, h
            q = (self._e(M, F_, dtype=torch.uint8), self._e(M, F_ // 32, dtype=torch.uint8))
            h = self._e(M, F_, dtype=BF16) if (tr and save) else False
            lin(a, wname, s.p(bname), act=ACT_SWISH, pre_out=z, out=h, out_bf16=True, q_out=q)
            return (h if h is not False else None), q

        def ln_in(xin, name, st, **kw):
            """LayerNorm feeding a Linear: bf16 output, or under fp8_gemm the MX-fp8 copy written by
            the LN kernel itself (bf16 kept only for the trained layers' weight gradients)."""
            if not fp8:
                y = self._e(M, D, dtype=BF16)
                sv[st] = self._ln(xin, name, eps, yb=y, **kw)
                return y, y
            y = self._e(M, D, dtype=BF16) if (tr and save) else None
            q = (self._e(M, D, dtype=torch.uint8), self._e(M, D // 32, dtype=torch.uint8))
            sv[st] = self._ln(xin, name, eps, yb=y, q8=q, **kw)
            return y, q

        def ln_in_out(name, tr_, **kw):
            """ln_in's outputs for a LayerNorm computed by a fused pair: (keyword set, a, ain)."""
            if not fp8:
                y = self._e(M, D, dtype=BF16)
                return dict(yb=y, **kw), y, y
            y = self._e(M, D, dtype=BF16) if (tr_ and save) else None
            q = (self._e(M, D, dtype=torch.uint8), self._e(M, D // 32, dtype=torch.uint8))
            return dict(yb=y, q8=q, **kw), y, q

        # -- FFN1 (half-step)
        if pre1 is not None:
            a1, a1in, sv["st1"] = pre1
        else:
            a1, a1in = ln_in(x, pre + "ffn1_layer_norm", "st1")
        z1 = self._e(M, F_, dtype=BF16) if save else None  # swish pre-activation, for backward only
        h1, h1in = ffn_in(a1in, pre + "ffn1.intermediate_dense.weight", pre + "ffn1.intermediate_dense.bias", z1)
        x1 = lin(h1in, pre + "ffn1.output_dense.weight", s.p(pre + "ffn1.output_dense.bias"), alpha=0.5,
                 residual=x)
        # -- relative-key MHSA
        a2, a2in = ln_in(x1, pre + "self_attn_layer_norm", "st2")
        qkv = lin(a2in, pre + "self_attn.linear_q.weight", s.fused(pre + "self_attn.linear_q.bias", 3, "p"), count=3,
                  out_bf16=True)
        o = self._e(M, D, dtype=BF16)
        o_lo = self._e(M, D, dtype=BF16) if save else None   # low half of O for the backward's delta
        lse = self._e(b * H * T)
        ops.attention_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], B=b, T=T, H=H, o=o, lse=lse, key_mask=mask32,
                          rel_E=s.w(pre + "self_attn.distance_embedding.weight"),
                          rel_left=c.left_max_position_embeddings, rel_right=c.right_max_position_embeddings,
                          scale=1.0 / math.sqrt(D // H), o_lo=o_lo)
        x2 = lin(o, pre + "self_attn.linear_out.weight", s.p(pre + "self_attn.linear_out.bias"), residual=x1)
        # -- convolution module
        a3, a3in = ln_in(x2, pre + "conv_module.layer_norm", "st3", row_scale=maskf)
        pw1 = lin(a3in, pre + "conv_module.pointwise_conv1.weight", None, out_bf16=True)
        cv = self._e(M, D, dtype=BF16)
        ops.glu_dwconv_fwd(pw1, s.p(pre + "conv_module.depthwise_conv.weight").view(D, -1), cv, b, T)
        sw, swin = ln_in(cv, pre + "conv_module.depthwise_layer_norm", "st4", act=ACT_SWISH)
        p_conv = c.conformer_conv_dropout if train else 0.0
        x3 = lin(swin, pre + "conv_module.pointwise_conv2.weight", None, residual=x2, drop_p=p_conv,
                 seed=_site_seed(seed, 1))
        # -- FFN2 (half-step) + final LN
        a5, a5in = ln_in(x3, pre + "ffn2_layer_norm", "st5")
        z2 = self._e(M, F_, dtype=BF16) if save else None
        h2, h2in = ffn_in(a5in, pre + "ffn2.intermediate_dense.weight", pre + "ffn2.intermediate_dense.bias", z2)
        x4 = lin(h2in, pre + "ffn2.output_dense.weight", s.p(pre + "ffn2.output_dense.bias"), alpha=0.5,
                 residual=x3)
        x5 = self._e(M, D)
        x5b = self._e(M, D, dtype=BF16) if want_bf16 else None
        pre_next = None
        if nxt is None:
            sv["st6"] = self._ln(x4, pre + "final_layer_norm", eps, y=x5, yb=x5b)
        else:
            # this final LN fused with layer nxt's FFN1 LN (x5 stays in registers for the second)
            prej = f"audio_encoder.encoder.layers.{nxt}.ffn1_layer_norm"
            trj = s.trainable_layer(f"audio_encoder.encoder.layers.{nxt}.ffn1_layer_norm.weight")
            second, a1j, a1inj = ln_in_out(prej, trj, gamma=s.p(prej + ".weight"), beta=s.p(prej + ".bias"), eps=eps)
            sv["st6"], st1j = ops.layernorm_fwd_pair(
                dict(x=x4, gamma=s.p(pre + "final_layer_norm.weight"), beta=s.p(pre + "final_layer_norm.bias"), eps=eps,
                     y=x5, yb=x5b), second)
            pre_next = (a1j, a1inj, st1j)
        sv.update(x=x, z1=z1, x1=x1, qkv=qkv, o=o, o_lo=o_lo, lse=lse, x2=x2, pw1=pw1, cv=cv, x3=x3, z2=z2, x4=x4, p_conv=p_conv)
        if tr:
            sv.update(a1=a1, h1=h1, a2=a2, a3=a3, sw=sw, a5=a5, h2=h2)
        return x5, x5b, sv, pre_next

    def _ln_bwd_kw(self, x, stats, name, **kw):
        """layernorm_bwd keyword set of the named LN (the pair kernels' argument form)."""
        return dict(x=x, mean=stats[0], rstd=stats[1], gamma=self.s.p(name + ".weight"), beta=self.s.p(name + ".bias"),
                    dgamma=self.s.g(name + ".weight"), dbeta=self.s.g(name + ".bias"), **kw)

    def _conformer_bwd(self, i, sv, dx5, b, T, maskf, mask32, pending=None):
        """Backward of one Conformer layer.  pending: the FFN1-LN backward of the layer above
        (keyword set, dy included), fused here with this layer's final-LN backward; dx5 is then
        None.  -> (d input or None, this layer's own FFN1-LN backward as a pending keyword set
        when fusion is on, else None)."""
        c = self.acfg
        s = self.s
        pre = f"audio_encoder.encoder.layers.{i}."
        M, D, F_ = sv["x4"].shape[0], c.hidden_size, c.intermediate_size
        H = c.num_attention_heads
        tr = sv["tr"]
        # final LN
        dx4 = self._e(M, D)
        dx4b = self._e(M, D, dtype=BF16)
        if pending is None:
            self._ln_bwd(dx5, sv["x4"], sv["st6"], pre + "final_layer_norm", dx=dx4, dxb=dx4b, out_scale=0.5,
                         dsum=s.g(pre + "ffn2.output_dense.bias"))
        else:
            ops.layernorm_bwd_pair(self._ln_bwd_kw(sv["x4"], sv["st6"], pre + "final_layer_norm", dx=dx4, dxb=dx4b,
                                                   out_scale=0.5, dsum=s.g(pre + "ffn2.output_dense.bias")), pending)
        # FFN2
        dz2 = self._dx(dx4b, pre + "ffn2.output_dense.weight", act=ACT_SWISH_BWD, z=sv["z2"],
                            out_bf16=True, colsum=s.g(pre + "ffn2.intermediate_dense.bias"))
        if tr:
            self._dw(dx4b, sv["h2"], pre + "ffn2.output_dense.weight")
        # dX GEMMs feeding an LN backward leave bf16 (as under the reference's bf16 autocast, whose
        # Linear backward returns a bf16 input gradient); the residual-stream gradient stays fp32
        da5 = self._dx(dz2, pre + "ffn2.intermediate_dense.weight", out_bf16=True)
        if tr:
            self._dw(dz2, sv["a5"], pre + "ffn2.intermediate_dense.weight")
        del dz2
        dx3 = self._e(M, D)
        dx3b = self._e(M, D, dtype=BF16)
        self._ln_bwd(da5, sv["x3"], sv["st5"], pre + "ffn2_layer_norm", dres=dx4, dx=dx3, dxb=dx3b,
                     drop_p=sv["p_conv"], seed=_site_seed(sv["seed"], 1))
        del da5, dx4, dx4b
        # conv module
        dsw = self._dx(dx3b, pre + "conv_module.pointwise_conv2.weight", out_bf16=True)
        if tr:
            self._dw(dx3b, sv["sw"], pre + "conv_module.pointwise_conv2.weight")
        dcv = self._e(M, D, dtype=BF16)
        self._ln_bwd(dsw, sv["cv"], sv["st4"], pre + "conv_module.depthwise_layer_norm", act=ACT_SWISH, dxb=dcv)
        del dsw
        dpw1 = self._e(M, 2 * D, dtype=BF16)
        gdw = s.g(pre + "conv_module.depthwise_conv.weight")
        ops.glu_dwconv_bwd(sv["pw1"], s.p(pre + "conv_module.depthwise_conv.weight").view(D, -1), dcv, dpw1,
                           None if gdw is None else gdw.view(D, -1), b, T)
        del dcv
        da3 = self._dx(dpw1, pre + "conv_module.pointwise_conv1.weight", out_bf16=True)
        if tr:
            self._dw(dpw1, sv["a3"], pre + "conv_module.pointwise_conv1.weight")
        del dpw1
        dx2 = self._e(M, D)
        dx2b = self._e(M, D, dtype=BF16)
        self._ln_bwd(da3, sv["x2"], sv["st3"], pre + "conv_module.layer_norm", row_scale=maskf, dres=dx3, dx=dx2,
                     dxb=dx2b, dsum=s.g(pre + "self_attn.linear_out.bias"))
        del da3, dx3, dx3b
        # attention
        do = self._dx(dx2b, pre + "self_attn.linear_out.weight", out_bf16=True)
        if tr:
            self._dw(dx2b, sv["o"], pre + "self_attn.linear_out.weight")
        del dx2b
        qkv = sv["qkv"]
        dqkv = self._e(M, 3 * D, dtype=BF16)
        delta = self._e(b * H * T)
        gE = s.g(pre + "self_attn.distance_embedding.weight")
        gwork = self._e(b * H * T * 80) if gE is not None else None
        ops.attention_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], sv["o"], sv["lse"], do, dqkv[:, :D],
                          dqkv[:, D:2 * D], dqkv[:, 2 * D:], B=b, T=T, H=H, delta=delta, key_mask=mask32,
                          rel_E=s.w(pre + "self_attn.distance_embedding.weight"),
                          rel_left=c.left_max_position_embeddings, rel_right=c.right_max_position_embeddings,
                          scale=1.0 / math.sqrt(D // H), dE=gE, gwork=gwork, o_lo=sv["o_lo"])
        del do, delta, gwork
        da2 = self._dx(dqkv, pre + "self_attn.linear_q.weight", 3, out_bf16=True)
        if tr:
            self._dw(dqkv, sv["a2"], pre + "self_attn.linear_q.weight", fused=3)
            self._db(dqkv, pre + "self_attn.linear_q.bias", fused=3)
        del dqkv
        dx1 = self._e(M, D)
        dx1b = self._e(M, D, dtype=BF16)
        self._ln_bwd(da2, sv["x1"], sv["st2"], pre + "self_attn_layer_norm", dres=dx2, dx=dx1, dxb=dx1b,
                     out_scale=0.5, dsum=s.g(pre + "ffn1.output_dense.bias"))
        del da2, dx2
        # FFN1
        dz1 = self._dx(dx1b, pre + "ffn1.output_dense.weight", act=ACT_SWISH_BWD, z=sv["z1"],
                            out_bf16=True, colsum=s.g(pre + "ffn1.intermediate_dense.bias"))
        if tr:
            self._dw(dx1b, sv["h1"], pre + "ffn1.output_dense.weight")
        da1 = self._dx(dz1, pre + "ffn1.intermediate_dense.weight", out_bf16=True)
        if tr:
            self._dw(dz1, sv["a1"], pre + "ffn1.intermediate_dense.weight")
        del dz1
        kw = self._ln_bwd_kw(sv["x"], sv["st1"], pre + "ffn1_layer_norm", dy=da1, dres=dx1)
        if self.ln_pair:
            return None, kw
        dx0 = self._e(M, D)
        ops.layernorm_bwd(dx=dx0, **kw)
        return dx0, None

    def _flush_ln(self, pending):
        """Run a pending FFN1-LN backward on its own -> its input gradient."""
        dx0 = self._e(*pending["x"].shape)
        ops.layernorm_bwd(dx=dx0, **pending)
        return dx0

    def audio_backward(self, dh, ctx, layers_done=None):
        """layers_done() is called once every trainable Conformer layer's gradients are final
        (after the lowest trainable layer), so their all-reduce overlaps the frozen layers."""
        if self.raw_audio:
            from . import wav2vec2
            return wav2vec2.backward(self, dh, ctx, layers_done)
        c = self.acfg
        b, T = ctx["a_b"], ctx["a_T"]
        maskf, mask32 = ctx["a_maskf"], ctx["a_mask32"]
        lo = next((i for i in range(c.num_hidden_layers)
                   if self.s.trainable_layer(f"audio_encoder.encoder.layers.{i}.ffn1_layer_norm.weight")), None)
        dx = dh
        pending = None
        for i in reversed(range(c.num_hidden_layers)):
            sv = ctx["a_layers"][i]
            if sv is not None:
                dx, pending = self._conformer_bwd(i, sv, dx, b, T, maskf, mask32, pending)
                ctx["a_layers"][i] = None
            if i == lo:
                # the lowest trainable layer's FFN1-LN gradients must be final before its sync;
                # flushed on every micro-batch (not only the one that syncs), so a micro-batch's
                # gradients never depend on its place in the accumulation window (the single and
                # pair LN kernels agree only to fp32 rounding)
                if pending is not None:
                    dx, pending = self._flush_ln(pending), None
                if layers_done is not None:
                    layers_done()
        if pending is not None:
            dx = self._flush_ln(pending)
        s = self.s
        if ctx.get("a_spec") is not None:  # SpecAugment rows: gradient to masked_spec_embed, not the projection
            ops.spec_mask_bwd(dx, ctx["a_spec"], maskf, s.g("audio_encoder.masked_spec_embed"))
        # feature projection: x = mask * (LN(feats) W^T + b)
        gW = s.g("audio_encoder.feature_projection.projection.weight")
        if gW is not None:
            M = dx.shape[0]
            # the forward's masked_fill (row_scale) multiplies dY row-wise
            _lib.call("ste_scale_rows", dx.data_ptr(), maskf.data_ptr(), M, c.hidden_size, dx.stride(0),
                      _lib.stream_ptr())
            dxb = ops.cast_bf16(dx, self._e(M, c.hidden_size, dtype=BF16))
            self._dw(dxb, ctx["a_a0"], "audio_encoder.feature_projection.projection.weight")
            self._db(dxb, "audio_encoder.feature_projection.projection.bias")
            if s.g("audio_encoder.feature_projection.layer_norm.weight") is not None:
                da0 = ops.linear_dx(dxb, s.w("audio_encoder.feature_projection.projection.weight"))
                self._ln_bwd(da0, ctx["a_xin"], ctx["a_st0"], "audio_encoder.feature_projection.layer_norm")

    # ================================================================= text
    def text_forward(self, ids, mask_i64, train, base_seed, ctx, save=True):
        c = self.tcfg
        s = self.s
        nb, L = ids.shape
        M, D = nb * L, c.hidden_size
        mask32 = self._e(M, dtype=torch.int32)
        _lib.call("ste_mask_i64_to_f32", mask_i64.data_ptr(), None, mask32.data_ptr(), M, _lib.stream_ptr())
        emb = self._e(M, D)
        pos_ids = self._e(M, dtype=torch.int32)
        ops.text_embed_fwd(ids, c.pad_token_id, s.p("text_encoder.embeddings.word_embeddings.weight"),
                           s.p("text_encoder.embeddings.position_embeddings.weight"),
                           s.p("text_encoder.embeddings.token_type_embeddings.weight"), emb, pos_ids)
        hp = c.hidden_dropout_prob if train else 0.0
        ap = c.attention_probs_dropout_prob if train else 0.0
        x = self._e(M, D)
        xb = self._e(M, D, dtype=BF16)
        st = self._ln(emb, "text_encoder.embeddings.LayerNorm", c.layer_norm_eps, y=x, yb=xb, drop_p=hp,
                      seed=_site_seed(base_seed, 1))
        ctx.update(t_nb=nb, t_L=L, t_mask32=mask32, t_ids=ids, t_emb=emb, t_pos=pos_ids, t_st=st, t_hp=hp, t_ap=ap,
                   t_seed=base_seed)
        layers = []
        for i in range(c.num_hidden_layers):
            x, xb, sv = self._xlmr_fwd(i, x, xb, nb, L, mask32, hp, ap, _site_seed(base_seed, 10 + i), save)
            layers.append(sv if save else None)
        ctx["t_layers"] = layers
        return x, xb

    def _xlmr_fwd(self, i, x, xb, nb, L, mask32, hp, ap, seed, save=True):
        return self._postln_fwd(self.tcfg, XLMR_NAMES, i, x, xb, nb, L, mask32, hp, ap, seed, save)

    def _xlmr_bwd(self, i, sv, dx2, nb, L, mask32, hp, ap):
        return self._postln_bwd(self.tcfg, XLMR_NAMES, i, sv, dx2, nb, L, mask32, hp, ap)

    def _postln_fwd(self, c, nm, i, x, xb, nb, L, mask32, hp, ap, seed, save=True, act_p=0.0):
        """One post-LN transformer layer: XLM-R (tf:…xlm_roberta…:186-398) and wav2vec2
        (tf:models/wav2vec2/modeling_wav2vec2.py:466-608) share the math
        LN(x + drop(O(attn(QKV x)))) -> LN(x1 + drop(W2·drop_act(gelu(W1 x1)))); `nm` maps the
        parameter names (XLMR_NAMES / W2V2_NAMES)."""
        s = self.s
        pre = nm["layer"].format(i=i)
        M, D, F_ = x.shape[0], c.hidden_size, c.intermediate_size
        H = c.num_attention_heads
        eps = c.layer_norm_eps
        tr = s.trainable_layer(pre + nm["q"] + ".weight")
        sv = {"tr": tr, "seed": seed, "act_p": act_p}
        qkv = ops.linear(xb, s.fused(pre + nm["q"] + ".weight", 3, "w"), s.fused(pre + nm["q"] + ".bias", 3, "p"),
                         out_bf16=True)
        o = self._e(M, D, dtype=BF16)
        o_lo = self._e(M, D, dtype=BF16) if save else None
        lse = self._e(nb * H * L)
        ops.attention_fwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], B=nb, T=L, H=H, o=o, lse=lse,
                          key_mask=mask32, scale=1.0 / math.sqrt(D // H), drop_p=ap, seed=_site_seed(seed, 1),
                          o_lo=o_lo)
        y1 = ops.linear(o, s.w(pre + nm["o"] + ".weight"), s.p(pre + nm["o"] + ".bias"),
                        residual=x, drop_p=hp, seed=_site_seed(seed, 2))
        x1 = self._e(M, D)
        x1b = self._e(M, D, dtype=BF16)
        sv["st1"] = self._ln(y1, pre + nm["ln1"], eps, y=x1, yb=x1b)
        zt = self._e(M, F_, dtype=BF16) if save else None  # GELU pre-activation, for backward only
        h = ops.linear(x1b, s.w(pre + nm["fi"] + ".weight"), s.p(pre + nm["fi"] + ".bias"),
                       act=ACT_GELU, pre_out=zt, out_bf16=True, drop_p=act_p, seed=_site_seed(seed, 4))
        y2 = ops.linear(h, s.w(pre + nm["fo"] + ".weight"), s.p(pre + nm["fo"] + ".bias"), residual=x1, drop_p=hp,
                        seed=_site_seed(seed, 3))
        x2 = self._e(M, D)
        x2b = self._e(M, D, dtype=BF16)
        sv["st2"] = self._ln(y2, pre + nm["ln2"], eps, y=x2, yb=x2b)
        sv.update(qkv=qkv, o=o, o_lo=o_lo, lse=lse, y1=y1, zt=zt, y2=y2)
        if tr:
            sv.update(xb=xb, x1b=x1b, h=h)
        return x2, x2b, sv

    def _postln_bwd(self, c, nm, i, sv, dx2, nb, L, mask32, hp, ap):
        s = self.s
        pre = nm["layer"].format(i=i)
        M, D = dx2.shape[0], c.hidden_size
        H = c.num_attention_heads
        tr = sv["tr"]
        seed = sv["seed"]
        dy2 = self._e(M, D)
        dy2b = self._e(M, D, dtype=BF16)
        self._ln_bwd(dx2, sv["y2"], sv["st2"], pre + nm["ln2"], dx=dy2, dxb=dy2b, drop_p=hp,
                     seed=_site_seed(seed, 3), dsum=s.g(pre + nm["fo"] + ".bias"))
        dzt = self._dx(dy2b, pre + nm["fo"] + ".weight", act=ACT_GELU_BWD, z=sv["zt"], out_bf16=True,
                       colsum=s.g(pre + nm["fi"] + ".bias"), drop_p=sv["act_p"], seed=_site_seed(seed, 4))
        if tr:
            self._dw(dy2b, sv["h"], pre + nm["fo"] + ".weight")
        del dy2b
        dx1 = self._dx(dzt, pre + nm["fi"] + ".weight", residual=dy2)
        if tr:
            self._dw(dzt, sv["x1b"], pre + nm["fi"] + ".weight")
        del dzt, dy2
        dy1 = self._e(M, D)
        dy1b = self._e(M, D, dtype=BF16)
        self._ln_bwd(dx1, sv["y1"], sv["st1"], pre + nm["ln1"], dx=dy1, dxb=dy1b, drop_p=hp,
                     seed=_site_seed(seed, 2), dsum=s.g(pre + nm["o"] + ".bias"))
        del dx1
        do = self._dx(dy1b, pre + nm["o"] + ".weight", out_bf16=True)
        if tr:
            self._dw(dy1b, sv["o"], pre + nm["o"] + ".weight")
        del dy1b
        qkv = sv["qkv"]
        dqkv = self._e(M, 3 * D, dtype=BF16)
        delta = self._e(nb * H * L)
        ops.attention_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], sv["o"], sv["lse"], do, dqkv[:, :D],
                          dqkv[:, D:2 * D], dqkv[:, 2 * D:], B=nb, T=L, H=H, delta=delta, key_mask=mask32,
                          scale=1.0 / math.sqrt(D // H), drop_p=ap, seed=_site_seed(seed, 1), o_lo=sv["o_lo"])
        del do, delta
        dx0 = self._dx(dqkv, pre + nm["q"] + ".weight", 3, residual=dy1)
        if tr:
            self._dw(dqkv, sv["xb"], pre + nm["q"] + ".weight", fused=3)
            self._db(dqkv, pre + nm["q"] + ".bias", fused=3)
        return dx0

    def text_backward(self, dh, ctx):
        c = self.tcfg
        s = self.s
        nb, L = ctx["t_nb"], ctx["t_L"]
        dx = dh
        for i in reversed(range(c.num_hidden_layers)):
            dx = self._xlmr_bwd(i, ctx["t_layers"][i], dx, nb, L, ctx["t_mask32"], ctx["t_hp"], ctx["t_ap"])
            ctx["t_layers"][i] = None
        gw = s.g("text_encoder.embeddings.word_embeddings.weight")
        gp = s.g("text_encoder.embeddings.position_embeddings.weight")
        gt = s.g("text_encoder.embeddings.token_type_embeddings.weight")
        ln_needed = any(g is not None for g in (gw, gp, gt, s.g("text_encoder.embeddings.LayerNorm.weight")))
        if not ln_needed:
            return
        demb = self._e(dx.shape[0], c.hidden_size)
        self._ln_bwd(dx, ctx["t_emb"], ctx["t_st"], "text_encoder.embeddings.LayerNorm", dx=demb,
                     in_drop_p=ctx["t_hp"], in_seed=_site_seed(ctx["t_seed"], 1))
        if gw is not None or gp is not None or gt is not None:
            ops.text_embed_bwd(ctx["t_ids"], ctx["t_pos"], demb, c.pad_token_id, gw, gp, gt)

    # ================================================================ heads
    def _proj_fwd(self, name, xb, rows, train, seed, sv):
        """EnhancedProjection ref:66-99 on bf16 input rows -> (fp32 [rows,P], bf16 copy)."""
        s = self.s
        p_drop = self.m.dropout if train else 0.0
        zp = self._e(rows, s.slots[name + ".projection.0.weight"].shape[0], dtype=BF16)
        hb = ops.linear(xb, s.w(name + ".projection.0.weight"), s.p(name + ".projection.0.bias"), act=ACT_GELU,
                        pre_out=zp, out_bf16=True, drop_p=p_drop, seed=seed)
        y = ops.linear(hb, s.w(name + ".projection.3.weight"), s.p(name + ".projection.3.bias"))
        P = y.shape[1]
        out = self._e(rows, P)
        st = self._ln(y, name + ".projection.4", 1e-5, y=out)
        sv.update(xb=xb, zp=zp, hb=hb, y=y, st=st, p=p_drop, seed=seed)
        return out

    def _proj_bwd(self, name, sv, dout, dx_out):
        """returns nothing; writes d(input) into dx_out (fp32, +=)."""
        s = self.s
        rows, P = dout.shape
        dyb = self._e(rows, P, dtype=BF16)
        self._ln_bwd(dout, sv["y"], sv["st"], name + ".projection.4", dxb=dyb, dsum=s.g(name + ".projection.3.bias"))
        dz = ops.linear_dx(dyb, s.w(name + ".projection.3.weight"), act=ACT_GELU_BWD, z=sv["zp"], out_bf16=True,
                           drop_p=sv["p"], seed=sv["seed"], colsum=s.g(name + ".projection.0.bias"))
        self._dw(dyb, sv["hb"], name + ".projection.3.weight")
        ops.linear_dx(dz, s.w(name + ".projection.0.weight"), out=dx_out, beta=1.0)
        self._dw(dz, sv["xb"], name + ".projection.0.weight")

    def _pool_fwd(self, name, hb, mask32, nb, L, sv):
        """AttentivePooling ref:171-211 -> pooled fp32 [nb, H] and bf16 copy.  With
        use_attentive_pooling=False: text CLS row (ref:578-580) / audio masked mean (ref:621-636)."""
        s = self.s
        H = hb.shape[1]
        if not self.m.use_attentive_pooling:
            w = self._e(nb * L)
            pooled = self._e(nb, H)
            pooledb = self._e(nb, H, dtype=BF16)
            ops.mean_pool_fwd(hb, mask32, nb, L, name == "text_pooling", w, pooled, pooledb)
            sv.update(w=w)
            return pooled, pooledb
        t = ops.linear(hb, s.w(name + ".attention.0.weight"), s.p(name + ".attention.0.bias"), act=ACT_TANH,
                       out_bf16=True)
        w = self._e(nb * L)
        pooled = self._e(nb, H)
        pooledb = self._e(nb, H, dtype=BF16)
        ops.attn_pool_fwd(t, s.p(name + ".attention.2.weight").view(-1), s.p(name + ".attention.2.bias"), hb, mask32,
                          nb, L, w, pooled, pooledb)
        sv.update(t=t, w=w, hb=hb, mask=mask32)
        return pooled, pooledb

    def _pool_bwd(self, name, sv, dpooled, dh, nb, L):
        s = self.s
        if not self.m.use_attentive_pooling:
            ops.weighted_pool_bwd(sv["w"], dpooled, nb, L, dh)
            return
        t = sv["t"]
        dz = self._e(*t.shape, dtype=BF16)
        gw1 = s.g(name + ".attention.0.weight")
        dz_lo = self._e(*t.shape, dtype=BF16) if gw1 is not None else None
        gw2 = s.g(name + ".attention.2.weight")
        # Σ_l dscore_l = 0 makes the scorer's first-Linear gradients small differences of large
        # terms: the bias gradient is summed in fp32 by the kernel, the weight gradient runs on
        # dz = hi + lo (two GEMM passes)
        ops.attn_pool_bwd(t, s.p(name + ".attention.2.weight").view(-1), sv["hb"], sv["w"], dpooled, nb, L, dh, dz,
                          None if gw2 is None else gw2.view(-1), s.g(name + ".attention.2.bias"),
                          db1=s.g(name + ".attention.0.bias"), dz_lo=dz_lo, mask=sv["mask"])
        ops.linear_dx(dz, s.w(name + ".attention.0.weight"), out=dh, beta=1.0)
        self._dw(dz, sv["hb"], name + ".attention.0.weight")
        if dz_lo is not None:
            self._dw(dz_lo, sv["hb"], name + ".attention.0.weight")

    def heads_forward(self, th, thb, ah, ahb, train, base_seed, ctx):
        s = self.s
        m = self.m
        nb, L = ctx["t_nb"], ctx["t_L"]
        b = nb // 2
        ab, T = ctx["a_b"], ctx["a_T"]
        P = m.projection_dim
        hs = {}
        # pooling + projection
        tpool_sv, apool_sv, tproj_sv, aproj_sv = {}, {}, {}, {}
        tpooled, tpooledb = self._pool_fwd("text_pooling", thb, ctx["t_mask32"], nb, L, tpool_sv)
        apooled, apooledb = self._pool_fwd("audio_pooling", ahb, ctx["a_mask32"], ab, T, apool_sv)
        tcat = self._e(nb, 2 * P, dtype=BF16)   # [tproj | t_att] bf16, fusion GEMM input
        acat = self._e(b, 2 * P, dtype=BF16)
        tproj = self._proj_fwd("text_projection", tpooledb, nb, train, _site_seed(base_seed, 201), tproj_sv)
        aproj = self._proj_fwd("audio_projection", apooledb, ab, train, _site_seed(base_seed, 202), aproj_sv)
        tprojb =ops.cast_bf16(tproj, self._e(nb, P, dtype=BF16))
        aprojb = ops.cast_bf16(aproj, self._e(ab, P, dtype=BF16))
        hs.update(tpool=tpool_sv, apool=apool_sv, tproj=tproj_sv, aproj=aproj_sv, tprojb=tprojb, aprojb=aprojb)
        if m.use_cross_modal:
            p_x = m.dropout if train else 0.0
            # audio_seq_to_projection (identical for the pos and neg calls of ref:525-542: computed once)
            aseqb = ops.linear(ahb, s.w("audio_seq_to_projection.weight"), s.p("audio_seq_to_projection.bias"),
                               out_bf16=True)
            # text->audio: K/V over the audio sequence shared by pos and neg queries
            kva = ops.linear(aseqb, s.fused("text_to_audio_attention.key.weight", 2, "w"),
                             s.fused("text_to_audio_attention.key.bias", 2, "p"), out_bf16=True)
            qt = ops.linear(tprojb, s.w("text_to_audio_attention.query.weight"),
                            s.p("text_to_audio_attention.query.bias"))
            nh = m.xattn_heads
            probs_t = self._e(nb * nh * T)
            att_t = self._e(nb, P)
            seed_t = _site_seed(base_seed, 203)
            # pos rows, neg rows: one launch over the shared audio keys (each half keeps its own seed)
            ops.xattn_fwd(qt, kva[:, :P], kva[:, P:], ctx["a_mask32"], b, T, nh, probs_t, att_t,
                          (_site_seed(seed_t, 0), _site_seed(seed_t, 1)), drop_p=p_x)
            att_tb = ops.cast_bf16(att_t, self._e(nb, P, dtype=BF16))
            ops.linear(att_tb, s.w("text_to_audio_attention.out_proj.weight"),
                       s.p("text_to_audio_attention.out_proj.bias"), out=tcat[:, P:])
            _copy_bf16(tprojb, tcat[:, :P])
            # audio->text (pos call only: the neg call's audio output is discarded, ref:535)
            tseqb = ops.linear(thb[: b * L], s.w("text_seq_to_projection.weight"), s.p("text_seq_to_projection.bias"),
                               out_bf16=True)
            kvt = ops.linear(tseqb, s.fused("audio_to_text_attention.key.weight", 2, "w"),
                             s.fused("audio_to_text_attention.key.bias", 2, "p"), out_bf16=True)
            qa = ops.linear(aprojb, s.w("audio_to_text_attention.query.weight"),
                            s.p("audio_to_text_attention.query.bias"))
            probs_a = self._e(b * nh * L)
            att_a = self._e(b, P)
            seed_a = _site_seed(base_seed, 204)
            ops.xattn1_fwd(qa, kvt[:, :P], kvt[:, P:], ctx["t_mask32"][: b * L], b, L, nh, probs_a, att_a,
                           drop_p=p_x, seed=seed_a)
            att_ab = ops.cast_bf16(att_a, self._e(b, P, dtype=BF16))
            ops.linear(att_ab, s.w("audio_to_text_attention.out_proj.weight"),
                       s.p("audio_to_text_attention.out_proj.bias"), out_bf16=True, out=acat[:, P:])
            _copy_bf16(aprojb, acat[:, :P])
            # fusion Linear + LN
            yt = ops.linear(tcat, s.w("text_fusion.0.weight"), s.p("text_fusion.0.bias"))
            tfused = self._e(nb, P)
            st_t = self._ln(yt, "text_fusion.1", 1e-5, y=tfused)
            ya = ops.linear(acat, s.w("audio_fusion.0.weight"), s.p("audio_fusion.0.bias"))
            afused = self._e(b, P)
            st_a = self._ln(ya, "audio_fusion.1", 1e-5, y=afused)
            hs.update(aseqb=aseqb, kva=kva, qt=qt, probs_t=probs_t, att_tb=att_tb, seed_t=seed_t, p_x=p_x,
                      tseqb=tseqb, kvt=kvt, qa=qa, probs_a=probs_a, att_ab=att_ab, seed_a=seed_a, tcat=tcat,
                      acat=acat, yt=yt, st_t=st_t, ya=ya, st_a=st_a)
        else:
            tfused, afused = tproj, aproj[:b]
        align = None
        if m.use_word_alignment:
            align = self._align_fwd(th, thb[: b * L], ahb, b, L, T, ctx, train, _site_seed(base_seed, 205), hs)
        ctx["heads"] = hs
        return tfused, afused, align

    def heads_backward(self, d_tfused, d_afused, d_align, ctx, dth, dah):
        s = self.s
        m = self.m
        hs = ctx["heads"]
        nb, L = ctx["t_nb"], ctx["t_L"]
        b = nb // 2
        ab, T = ctx["a_b"], ctx["a_T"]
        P = m.projection_dim
        d_tproj = self._z(nb, P)
        d_aproj = self._z(ab, P)
        if d_align is not None and m.use_word_alignment:
            self._align_bwd(d_align, hs, ctx, dth, dah)
        if m.use_cross_modal:
            # fusion LNs + Linears
            dyt = self._e(nb, P, dtype=BF16)
            self._ln_bwd(d_tfused, hs["yt"], hs["st_t"], "text_fusion.1", dxb=dyt, dsum=s.g("text_fusion.0.bias"))
            dtcat = ops.linear_dx(dyt, s.w("text_fusion.0.weight"))
            self._dw(dyt, hs["tcat"], "text_fusion.0.weight")
            dya = self._e(b, P, dtype=BF16)
            self._ln_bwd(d_afused, hs["ya"], hs["st_a"], "audio_fusion.1", dxb=dya, dsum=s.g("audio_fusion.0.bias"))
            dacat = ops.linear_dx(dya, s.w("audio_fusion.0.weight"))
            self._dw(dya, hs["acat"], "audio_fusion.0.weight")
            _add_(d_tproj, dtcat[:, :P])
            _add_(d_aproj[:b], dacat[:, :P])
            nh = m.xattn_heads
            # ---- text->audio attention (pos + neg queries, shared audio K/V)
            datt = dtcat[:, P:].contiguous()
            dattb = ops.cast_bf16(datt, self._e(nb, P, dtype=BF16))
            dq_in = ops.linear_dx(dattb, s.w("text_to_audio_attention.out_proj.weight"))
            self._dw(dattb, hs["att_tb"], "text_to_audio_attention.out_proj.weight")
            self._db(datt, "text_to_audio_attention.out_proj.bias")
            dqt = self._e(nb, P)
            # dK/dV come out of the kernel in bf16 with their fp32 column sums (the fused key/value
            # bias gradient); the K/V input gradient leaves its GEMM in bf16 with the
            # audio_seq_to_projection bias gradient summed in the epilogue: no fp32 [ab*T, 2P]
            # zero-fill / accumulate / cast / column-sum passes
            dkvb = self._e(ab * T, 2 * P, dtype=BF16)
            ops.xattn_bwd(hs["qt"], hs["kva"][:, :P], hs["kva"][:, P:], hs["probs_t"], dq_in, b, T, nh, dqt,
                          dkvb[:, :P], dkvb[:, P:], (_site_seed(hs["seed_t"], 0), _site_seed(hs["seed_t"], 1)),
                          drop_p=hs["p_x"], colsum=s.fused("text_to_audio_attention.key.bias", 2, "g"),
                          mask=ctx["a_mask32"])
            dqtb = ops.cast_bf16(dqt, self._e(nb, P, dtype=BF16))
            ops.linear_dx(dqtb, s.w("text_to_audio_attention.query.weight"), out=d_tproj, beta=1.0)
            self._dw(dqtb, hs["tprojb"], "text_to_audio_attention.query.weight")
            self._db(dqt, "text_to_audio_attention.query.bias")
            daseqb = self._dx(dkvb, "text_to_audio_attention.key.weight", 2, out_bf16=True,
                              colsum=s.g("audio_seq_to_projection.bias"))
            self._dw(dkvb, hs["aseqb"], "text_to_audio_attention.key.weight", fused=2)
            del dkvb
            self._dx(daseqb, "audio_seq_to_projection.weight", out=dah, beta=1.0)
            self._dw(daseqb, ctx["_ahb"], "audio_seq_to_projection.weight")
            del daseqb
            # ---- audio->text attention (pos call)
            datta = dacat[:, P:].contiguous()
            dattab = ops.cast_bf16(datta, self._e(b, P, dtype=BF16))
            dqa_in = ops.linear_dx(dattab, s.w("audio_to_text_attention.out_proj.weight"))
            self._dw(dattab, hs["att_ab"], "audio_to_text_attention.out_proj.weight")
            self._db(datta, "audio_to_text_attention.out_proj.bias")
            dqa = self._e(b, P)
            dkvtb = self._e(b * L, 2 * P, dtype=BF16)
            ops.xattn1_bwd(hs["qa"], hs["kvt"][:, :P], hs["kvt"][:, P:], hs["probs_a"], dqa_in, b, L, nh, dqa,
                           dkvtb[:, :P], dkvtb[:, P:], drop_p=hs["p_x"], seed=hs["seed_a"],
                           colsum=s.fused("audio_to_text_attention.key.bias", 2, "g"), mask=ctx["t_mask32"][: b * L])
            dqab = ops.cast_bf16(dqa, self._e(b, P, dtype=BF16))
            ops.linear_dx(dqab, s.w("audio_to_text_attention.query.weight"), out=d_aproj[:b], beta=1.0)
            self._dw(dqab, hs["aprojb"], "audio_to_text_attention.query.weight")
            self._db(dqa, "audio_to_text_attention.query.bias")
            dtseqb = ops.linear_dx(dkvtb, s.fused("audio_to_text_attention.key.weight", 2, "w"), out_bf16=True,
                                   colsum=s.g("text_seq_to_projection.bias"))
            self._dw(dkvtb, hs["tseqb"], "audio_to_text_attention.key.weight", fused=2)
            ops.linear_dx(dtseqb, s.w("text_seq_to_projection.weight"), out=dth[: b * L], beta=1.0)
            self._dw(dtseqb, ctx["_thb"][: b * L], "text_seq_to_projection.weight")
        else:
            _add_(d_tproj, d_tfused)
            _add_(d_aproj[:b], d_afused)
        # projections
        dtpooled = self._z(nb, self.tcfg.hidden_size)
        dapooled = self._z(ab, self.acfg.hidden_size)
        self._proj_bwd("text_projection", hs["tproj"], d_tproj, dtpooled)
        self._proj_bwd("audio_projection", hs["aproj"], d_aproj, dapooled)
        # pooling
        self._pool_bwd("text_pooling", hs["tpool"], dtpooled, dth, nb, L)
        self._pool_bwd("audio_pooling", hs["apool"], dapooled, dah, ab, T)

    # ------------------------------------ standalone cross-modal attention (public API)
    def _mask32(self, mask_i64, n):
        m = self._e(n, dtype=torch.int32)
        _lib.call("ste_mask_i64_to_f32", mask_i64.contiguous().data_ptr(), None, m.data_ptr(), n, _lib.stream_ptr())
        return m

    def cross_forward(self, tproj, th, tmask, aproj, ah, amask, train, seed):
        """apply_cross_modal_attention (ref:643-682) for one call: text [b,P] + hidden [b,L,Ht],
        audio [b,P] + hidden [b,T,Ha] -> (text_fused, audio_fused) [b,P] fp32 and the saved
        context.  The fused training step shares one audio K/V between the pos and neg calls
        (heads_forward); this is the reference's per-call form behind the public method."""
        s = self.s
        m = self.m
        b, L, Ht = th.shape
        T, Ha = ah.shape[1], ah.shape[2]
        P = m.projection_dim
        nh = m.xattn_heads
        p_x = m.dropout if train else 0.0
        thb = ops.cast_bf16(th.contiguous(), self._e(b * L, Ht, dtype=BF16))
        ahb = ops.cast_bf16(ah.contiguous(), self._e(b * T, Ha, dtype=BF16))
        tprojb = ops.cast_bf16(tproj.contiguous(), self._e(b, P, dtype=BF16))
        aprojb = ops.cast_bf16(aproj.contiguous(), self._e(b, P, dtype=BF16))
        tm32 = self._mask32(tmask, b * L) if tmask is not None else None
        if amask is not None and self.raw_audio and amask.shape[-1] != T:
            # a sample-level wav2vec2 mask [b, N]: the frame mask of the conv stack
            from .wav2vec2 import frame_mask
            am32 = frame_mask(self.acfg, amask, b, amask.shape[-1], T, self.s.device)[1]
        else:
            am32 = self._mask32(amask, b * T) if amask is not None else None
        # text -> audio
        aseqb = ops.linear(ahb, s.w("audio_seq_to_projection.weight"), s.p("audio_seq_to_projection.bias"),
                           out_bf16=True)
        kva = ops.linear(aseqb, s.fused("text_to_audio_attention.key.weight", 2, "w"),
                         s.fused("text_to_audio_attention.key.bias", 2, "p"), out_bf16=True)
        qt = ops.linear(tprojb, s.w("text_to_audio_attention.query.weight"), s.p("text_to_audio_attention.query.bias"))
        probs_t, att_t = self._e(b * nh * T), self._e(b, P)
        seed_t, seed_a = _site_seed(seed, 1), _site_seed(seed, 2)
        ops.xattn1_fwd(qt, kva[:, :P], kva[:, P:], am32, b, T, nh, probs_t, att_t, drop_p=p_x, seed=seed_t)
        att_tb = ops.cast_bf16(att_t, self._e(b, P, dtype=BF16))
        tcat = self._e(b, 2 * P, dtype=BF16)
        ops.linear(att_tb, s.w("text_to_audio_attention.out_proj.weight"), s.p("text_to_audio_attention.out_proj.bias"),
                   out=tcat[:, P:])
        _copy_bf16(tprojb, tcat[:, :P])
        # audio -> text
        tseqb = ops.linear(thb, s.w("text_seq_to_projection.weight"), s.p("text_seq_to_projection.bias"),
                           out_bf16=True)
        kvt = ops.linear(tseqb, s.fused("audio_to_text_attention.key.weight", 2, "w"),
                         s.fused("audio_to_text_attention.key.bias", 2, "p"), out_bf16=True)
        qa = ops.linear(aprojb, s.w("audio_to_text_attention.query.weight"), s.p("audio_to_text_attention.query.bias"))
        probs_a, att_a = self._e(b * nh * L), self._e(b, P)
        ops.xattn1_fwd(qa, kvt[:, :P], kvt[:, P:], tm32, b, L, nh, probs_a, att_a, drop_p=p_x, seed=seed_a)
        att_ab = ops.cast_bf16(att_a, self._e(b, P, dtype=BF16))
        acat = self._e(b, 2 * P, dtype=BF16)
        ops.linear(att_ab, s.w("audio_to_text_attention.out_proj.weight"), s.p("audio_to_text_attention.out_proj.bias"),
                   out=acat[:, P:])
        _copy_bf16(aprojb, acat[:, :P])
        # fusion Linear + LN
        yt = ops.linear(tcat, s.w("text_fusion.0.weight"), s.p("text_fusion.0.bias"))
        tfused = self._e(b, P)
        st_t = self._ln(yt, "text_fusion.1", 1e-5, y=tfused)
        ya = ops.linear(acat, s.w("audio_fusion.0.weight"), s.p("audio_fusion.0.bias"))
        afused = self._e(b, P)
        st_a = self._ln(ya, "audio_fusion.1", 1e-5, y=afused)
        sv = dict(b=b, L=L, T=T, thb=thb, ahb=ahb, tprojb=tprojb, aprojb=aprojb, aseqb=aseqb, kva=kva, qt=qt,
                  probs_t=probs_t, att_tb=att_tb, seed_t=seed_t, tseqb=tseqb, kvt=kvt, qa=qa, probs_a=probs_a,
                  att_ab=att_ab, seed_a=seed_a, p_x=p_x, tcat=tcat, acat=acat, yt=yt, st_t=st_t, ya=ya, st_a=st_a,
                  am32=am32, tm32=tm32)
        return tfused, afused, sv

    def cross_backward(self, sv, d_tf, d_af):
        """-> (d text_projected [b,P], d text_hidden [b*L,Ht], d audio_projected [b,P],
        d audio_hidden [b*T,Ha]) fp32; parameter gradients += into the flat buffer."""
        s = self.s
        m = self.m
        b, L, T = sv["b"], sv["L"], sv["T"]
        P = m.projection_dim
        nh = m.xattn_heads
        Ht, Ha = sv["thb"].shape[1], sv["ahb"].shape[1]
        d_tproj, d_aproj = self._z(b, P), self._z(b, P)
        dth, dah = self._z(b * L, Ht), self._z(b * T, Ha)
        dyt = self._e(b, P, dtype=BF16)
        self._ln_bwd(d_tf.contiguous(), sv["yt"], sv["st_t"], "text_fusion.1", dxb=dyt, dsum=s.g("text_fusion.0.bias"))
        dtcat = ops.linear_dx(dyt, s.w("text_fusion.0.weight"))
        self._dw(dyt, sv["tcat"], "text_fusion.0.weight")
        dya = self._e(b, P, dtype=BF16)
        self._ln_bwd(d_af.contiguous(), sv["ya"], sv["st_a"], "audio_fusion.1", dxb=dya, dsum=s.g("audio_fusion.0.bias"))
        dacat = ops.linear_dx(dya, s.w("audio_fusion.0.weight"))
        self._dw(dya, sv["acat"], "audio_fusion.0.weight")
        _add_(d_tproj, dtcat[:, :P])
        _add_(d_aproj, dacat[:, :P])
        # text -> audio
        datt = dtcat[:, P:].contiguous()
        dattb = ops.cast_bf16(datt, self._e(b, P, dtype=BF16))
        dq_in = ops.linear_dx(dattb, s.w("text_to_audio_attention.out_proj.weight"))
        self._dw(dattb, sv["att_tb"], "text_to_audio_attention.out_proj.weight")
        self._db(datt, "text_to_audio_attention.out_proj.bias")
        dqt = self._e(b, P)
        dkv = self._z(b * T, 2 * P)
        ops.xattn1_bwd(sv["qt"], sv["kva"][:, :P], sv["kva"][:, P:], sv["probs_t"], dq_in, b, T, nh, dqt, dkv[:, :P],
                       dkv[:, P:], drop_p=sv["p_x"], seed=sv["seed_t"], mask=sv["am32"])
        dqtb = ops.cast_bf16(dqt, self._e(b, P, dtype=BF16))
        ops.linear_dx(dqtb, s.w("text_to_audio_attention.query.weight"), out=d_tproj, beta=1.0)
        self._dw(dqtb, sv["tprojb"], "text_to_audio_attention.query.weight")
        self._db(dqt, "text_to_audio_attention.query.bias")
        dkvb = ops.cast_bf16(dkv, self._e(b * T, 2 * P, dtype=BF16))
        daseq = self._dx(dkvb, "text_to_audio_attention.key.weight", 2)
        self._dw(dkvb, sv["aseqb"], "text_to_audio_attention.key.weight", fused=2)
        self._db(dkv, "text_to_audio_attention.key.bias", fused=2)
        daseqb = ops.cast_bf16(daseq, self._e(b * T, P, dtype=BF16))
        self._dx(daseqb, "audio_seq_to_projection.weight", out=dah, beta=1.0)
        self._dw(daseqb, sv["ahb"], "audio_seq_to_projection.weight")
        self._db(daseq, "audio_seq_to_projection.bias")
        # audio -> text
        datta = dacat[:, P:].contiguous()
        dattab = ops.cast_bf16(datta, self._e(b, P, dtype=BF16))
        dqa_in = ops.linear_dx(dattab, s.w("audio_to_text_attention.out_proj.weight"))
        self._dw(dattab, sv["att_ab"], "audio_to_text_attention.out_proj.weight")
        self._db(datta, "audio_to_text_attention.out_proj.bias")
        dqa = self._e(b, P)
        dkvt = self._z(b * L, 2 * P)
        ops.xattn1_bwd(sv["qa"], sv["kvt"][:, :P], sv["kvt"][:, P:], sv["probs_a"], dqa_in, b, L, nh, dqa,
                       dkvt[:, :P], dkvt[:, P:], drop_p=sv["p_x"], seed=sv["seed_a"], mask=sv["tm32"])
        dqab = ops.cast_bf16(dqa, self._e(b, P, dtype=BF16))
        ops.linear_dx(dqab, s.w("audio_to_text_attention.query.weight"), out=d_aproj, beta=1.0)
        self._dw(dqab, sv["aprojb"], "audio_to_text_attention.query.weight")
        self._db(dqa, "audio_to_text_attention.query.bias")
        dkvtb = ops.cast_bf16(dkvt, self._e(b * L, 2 * P, dtype=BF16))
        dtseq = ops.linear_dx(dkvtb, s.fused("audio_to_text_attention.key.weight", 2, "w"))
        self._dw(dkvtb, sv["tseqb"], "audio_to_text_attention.key.weight", fused=2)
        self._db(dkvt, "audio_to_text_attention.key.bias", fused=2)
        dtseqb = ops.cast_bf16(dtseq, self._e(b * L, P, dtype=BF16))
        ops.linear_dx(dtseqb, s.w("text_seq_to_projection.weight"), out=dth, beta=1.0)
        self._dw(dtseqb, sv["thb"], "text_seq_to_projection.weight")
        self._db(dtseq, "text_seq_to_projection.bias")
        return d_tproj, dth, d_aproj, dah

    # ------------------------------------------------------- word alignment
    def _align_fwd(self, th, thb_pos, ahb, b, L, T, ctx, train, seed, hs):
        from .align import align_forward
        return align_forward(self, th, thb_pos, ahb, b, L, T, ctx, train, seed, hs)

    def _align_bwd(self, d_align, hs, ctx, dth, dah):
        from .align import align_backward
        align_backward(self, d_align, hs, ctx, dth, dah)

    # ============================================================== full step
    def forward(self, batch, train: bool, save: bool = True):
        """compute_pos_neg_embeddings (ref:502-565) -> (tp_fused, tn_fused, a_fused, align, ctx).
        save=False (forward-only evaluation, ref:1165-1284 under no_grad): no encoder layer keeps
        its activations, so each layer's buffers return to the allocator as the next one runs, and
        the FFN GEMMs skip the pre-activation copies only backward reads."""
        ctx = Ctx()
        base_seed = int(torch.randint(0, 2**62, (1,)).item()) if train else 0
        ids = torch.cat([batch["input_ids_pos"], batch["input_ids_neg"]], 0)
        tmask = torch.cat([batch["attention_mask_pos"], batch["attention_mask_neg"]], 0).contiguous()
        ctx["_tmask_i64"] = tmask  # rows [0, b) = positive transcripts (alignment head's text mask)
        side = self._side_stream()
        if side is not None:  # text encoder on the side stream, audio encoder on the main stream
            main = torch.cuda.current_stream(self.s.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                th, thb = self.text_forward(ids.contiguous(), tmask, train, _site_seed(base_seed, 2), ctx, save)
        else:
            th, thb = self.text_forward(ids.contiguous(), tmask, train, _site_seed(base_seed, 2), ctx, save)
        amask = batch.get("attention_mask_audio")
        ah, ahb = self.audio_forward(batch["input_values"].contiguous(),
                                     None if amask is None else amask.contiguous(), train, _site_seed(base_seed, 3),
                                     ctx, save)
        if side is not None:
            main.wait_stream(side)
        ctx["_thb"], ctx["_ahb"] = thb, ahb
        tf, af, align = self.heads_forward(th, thb, ah, ahb, train, _site_seed(base_seed, 4), ctx)
        b = batch["input_ids_pos"].shape[0]
        return tf[:b], tf[b:], af, align, ctx

    def backward(self, ctx, d_tp, d_tn, d_af, d_align, stage_done=None):
        """Backward of the whole step.  stage_done(name) is called once the gradients of a
        parameter block are final (GradSync.STAGES order: "heads", "audio_layers", "audio",
        "text"), so a data-parallel
        caller can start their collective while the rest of the backward runs."""
        nb = ctx["t_nb"]
        d_tf = self._e(nb, self.m.projection_dim)
        _copy_f32(d_tp, d_tf[: nb // 2])
        _copy_f32(d_tn, d_tf[nb // 2:])
        dth = self._z(nb * ctx["t_L"], self.tcfg.hidden_size)
        dah = self._z(ctx["a_b"] * ctx["a_T"], self.acfg.hidden_size)
        self.heads_backward(d_tf, d_af, d_align, ctx, dth, dah)
        ctx.pop("heads", None)
        if stage_done:
            stage_done("heads")
        side = self._side_stream()
        if side is not None:  # text backward on the side stream, concurrent with the audio backward
            main = torch.cuda.current_stream(self.s.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.text_backward(dth, ctx)
            self.audio_backward(dah, ctx, (lambda: stage_done("audio_layers")) if stage_done else None)
            main.wait_stream(side)
            del dah
            if stage_done:
                stage_done("audio")
                stage_done("text")
        else:
            self.audio_backward(dah, ctx, (lambda: stage_done("audio_layers")) if stage_done else None)
            del dah
            if stage_done:
                stage_done("audio")
            self.text_backward(dth, ctx)
            if stage_done:
                stage_done("text")
        ctx.clear()


def _copy_bf16(src, dst):
    """dst[:] = src (strided 2-D views) on the ste_copy2d kernel."""
    ops.copy2d(dst, src)


def _copy_f32(src, dst):
    ops.copy2d(dst, src)


def _add_(dst, src):
    ops.axpby(dst, src, 1.0, 1.0)
