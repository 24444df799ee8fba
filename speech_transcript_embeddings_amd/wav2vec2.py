"""wav2vec2 raw-waveform audio encoder on the HIP kernels.

EnhancedAudioTextModel(audio_model_name="facebook/wav2vec2-base") — the reference's
encode_audio (ref:training/trainer_unfreeze.py:587-641) first tries
``audio_encoder(input_values=..., attention_mask=...)``, which for a Wav2Vec2Model takes RAW
16 kHz samples [B, N].  transformers' forward (tf = transformers/models/wav2vec2/
modeling_wav2vec2.py) restated as an explicit schedule:

  feature_extractor  :382-419  conv0 (1->512, k10 s5) + GroupNorm(512) + GELU    ste_w2v_conv0_fwd,
                               ste_w2v_gn_fwd;  conv1..6 (k3/k2, s2) + GELU: ste_gemm on a
                               strided VIEW of the previous output (row stride s·C, K = k·C)
  frame mask         :997-1036 ste_w2v_frame_mask
  feature_projection :422-434  LayerNorm(512) + Linear(512->768) + dropout       layernorm / gemm
  SpecAugment        :1272-1316 (training) spec_mask (specaug.py, as for w2v-bert)
  encoder prologue   :678-692  x[~mask] = 0; x + GELU(pos_conv(x)); LayerNorm; dropout
                     pos_conv  :326-379 weight-normed grouped Conv1d(768, 768, 128, pad 64, 16 groups),
                               SamePad: ONE batched ste_gemm (batch = groups) over the padded
                               group-major copy (ste_w2v_pos_pack), implicit im2col row stride D/G
  layers             :575-608  post-LN transformer layers = Engine._postln_fwd (shared with XLM-R)

Backward is the reverse schedule: dX of each strided conv is a plain GEMM into im2col space
folded back by ste_w2v_conv_fold (which also applies GELU'), dW is a per-clip batched GEMM on
the same strided views summed by ste_w2v_slab_sum; the positional conv's dX is the same
grouped GEMM with reversed taps (wf), its dW one batched GEMM whose k-major operands are the
padded copies (row stride D/G again), then the weight-norm backward.

Masks: with an attention mask the frame mask follows the conv output lengths (padded frames
zeroed before the positional conv and excluded as attention keys, as in transformers).  The
reference itself cannot run that case (its pooling applies the SAMPLE-level mask to frame-level
hidden states); with attention_mask=None — what wav2vec2-base's processor returns —
both agree and every frame is valid.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib, ops
from ._lib import ptr

BF16, F32 = torch.bfloat16, torch.float32
FE = "audio_encoder.feature_extractor.conv_layers."
PC = "audio_encoder.encoder.pos_conv_embed.conv."


def _s():
    return _lib.stream_ptr()


def frame_mask(cfg, mask_i64, B, N, Tf, device, maskf=None, mask32=None):
    """Frame-level masks [B*Tf] (float, int32) from a sample-level mask [B, N] (None = all valid)."""
    maskf = torch.empty(B * Tf, device=device, dtype=F32) if maskf is None else maskf
    mask32 = torch.empty(B * Tf, device=device, dtype=torch.int32) if mask32 is None else mask32
    n = len(cfg.conv_kernel)
    ks = (C.c_int * n)(*cfg.conv_kernel)
    ss = (C.c_int * n)(*cfg.conv_stride)
    m = None if mask_i64 is None else mask_i64.contiguous()
    _lib.call("ste_w2v_frame_mask", ptr(m), B, N, Tf, n, ks, ss, ptr(maskf), ptr(mask32), _s())
    return maskf, mask32


def wave_normalize(wave, lengths=None, pad=0.0):
    """Wav2Vec2FeatureExtractor(do_normalize=True) on the GPU: per-clip zero mean / unit variance
    over each clip's samples, `pad` after them.  wave fp32 [B, N]."""
    B, N = wave.shape
    out = torch.empty(B, N, device=wave.device, dtype=F32)
    lens = None if lengths is None else lengths.to(device=wave.device, dtype=torch.int32).contiguous()
    _lib.call("ste_w2v_wave_norm", ptr(wave), wave.stride(0), ptr(lens), B, N, float(pad), ptr(out), _s())
    return out


def _conv_weight(e, l, cin, k):
    """Conv1d weight [Co, Ci, k] (bf16 shadow) -> the GEMM's B operand [Co, k·Ci] (bf16)."""
    w = e.s.w(FE + f"{l}.conv.weight")
    co = w.shape[0]
    out = e._e(co, k * cin, dtype=BF16)
    _lib.call("ste_w2v_perm12", ptr(w), ptr(out), co, cin, k, 0, _s())
    return out


def forward(e, wave, mask_i64, train, base_seed, ctx, save=True, lengths=None):
    """Raw waveform fp32 [B, N] (+ sample mask [B, N] or None) -> (hidden fp32 [B*T, D], bf16 copy).
    lengths: host list of each clip's valid samples (SpecAugment's span sampling without a sync)."""
    from .engine import W2V2_NAMES, _site_seed
    c = e.acfg
    s = e.s
    if wave.dim() != 2:
        raise ValueError(f"wav2vec2 input_values must be raw samples [B, N], got shape {tuple(wave.shape)}")
    wave = wave.float().contiguous()
    B, N = wave.shape
    Ts = c.frames(N)
    if min(Ts[1:]) <= 0:
        raise ValueError(f"waveform of {N} samples is shorter than the conv stack's receptive field")
    T = Ts[-1]
    D = c.hidden_size
    M = B * T
    maskf, mask32 = frame_mask(c, mask_i64, B, N, T, wave.device)
    # ---- conv0 + GroupNorm + GELU
    C0, K0, S0 = c.conv_dim[0], c.conv_kernel[0], c.conv_stride[0]
    T0 = Ts[1]
    y0 = e._e(B * T0, C0)
    _lib.call("ste_w2v_conv0_fwd", ptr(wave), wave.stride(0), ptr(s.p(FE + "0.conv.weight")), B, N, T0, C0, K0, S0,
              ptr(y0), _s())
    gn_mean, gn_rstd = e._e(B * C0), e._e(B * C0)
    h = e._e(B * T0, C0, dtype=BF16)
    nwork = int(_lib.fn("ste_w2v_gn_work")(B, T0, C0, 1))
    work = e._e(nwork)
    _lib.call("ste_w2v_gn_fwd", ptr(y0), ptr(s.p(FE + "0.layer_norm.weight")), ptr(s.p(FE + "0.layer_norm.bias")),
              B, T0, C0, 1e-5, ptr(gn_mean), ptr(gn_rstd), ptr(h), ptr(work), nwork, _s())
    del work
    convs = [dict(h=h)]
    # ---- conv1.. : GEMM on the strided view of the previous output, GELU epilogue
    nl = len(c.conv_dim)
    for l in range(1, nl):
        cin, cout, k, st = c.conv_dim[l - 1], c.conv_dim[l], c.conv_kernel[l], c.conv_stride[l]
        Ti, To = Ts[l], Ts[l + 1]
        wr = _conv_weight(e, l, cin, k)
        a = torch.as_strided(h, (To, k * cin), (st * cin, 1))
        z = e._e(B * To, cout, dtype=BF16) if save else None
        last = l == nl - 1
        out = e._e(B * To, cout, dtype=F32 if last else BF16)
        ops.gemm(a, wr, M=To, N=cout, K=k * cin, batch=B, stride_a=Ti * cin, stride_c=To * cout, out=out,
                 act=_lib.ACT_GELU, pre_out=z)
        convs.append(dict(z=z, wr=wr, h=None if last else out))
        h = out
    # ---- feature projection (+ dropout), SpecAugment, padded frames zeroed
    a0 = e._e(M, c.conv_dim[-1], dtype=BF16)
    st0 = e._ln(h, "audio_encoder.feature_projection.layer_norm", c.layer_norm_eps, yb=a0)
    p_fp = c.feat_proj_dropout if train else 0.0
    seed_fp = _site_seed(base_seed, 7)
    x = ops.linear(a0, s.w("audio_encoder.feature_projection.projection.weight"),
                   s.p("audio_encoder.feature_projection.projection.bias"), row_scale=maskf, drop_p=p_fp, seed=seed_fp)
    spec = None
    if train and getattr(e.m, "spec_augment", False) and c.mask_time_prob > 0:
        from .specaug import compute_mask_indices, upload_mask
        if lengths is not None:   # host sample counts -> frames (the conv stack's output lengths)
            lens = [max(0, c.frames(int(n))[-1]) for n in lengths]
        else:                     # only a device mask: one device->host sync
            lens = maskf.view(B, T).sum(-1).to(torch.int64).tolist()
        sm = compute_mask_indices((B, T), c.mask_time_prob, c.mask_time_length, lens, c.mask_time_min_masks)
        spec = upload_mask(sm, s.device)
        ops.spec_mask_fwd(x, spec, maskf, s.p("audio_encoder.masked_spec_embed"))
    # ---- positional conv + residual + encoder LayerNorm (+ dropout)
    G, Kp = c.num_conv_pos_embedding_groups, c.num_conv_pos_embeddings
    Cg = D // G
    Tp = T + Kp - 1
    v, g = s.p(PC + "parametrizations.weight.original1"), s.p(PC + "parametrizations.weight.original0")
    norms = e._e(Kp)
    wr = e._e(G * Cg * Kp * Cg, dtype=BF16)
    wf = e._e(G * Cg * Kp * Cg, dtype=BF16)
    _lib.call("ste_w2v_wnorm_fwd", ptr(v), ptr(g), D, Cg, Kp, ptr(norms), ptr(wr), ptr(wf), _s())
    seg = B * Tp + Kp
    xp = e._e(G * seg * Cg, dtype=BF16)
    _lib.call("ste_w2v_pos_pack", ptr(x), B, T, D, G, Kp, Kp // 2, ptr(xp), _s())
    cpad = e._e(B * Tp, D)
    _pos_gemm(xp, wr, cpad, B * Tp, G, Cg, Kp, seg)
    xe = e._e(M, D)
    _lib.call("ste_w2v_pos_elem", 0, ptr(cpad), ptr(s.p(PC + "bias")), ptr(x), None, B, T, D, Tp, ptr(xe), _s())
    hp = c.hidden_dropout if train else 0.0
    ap = c.attention_dropout if train else 0.0
    act_p = c.activation_dropout if train else 0.0
    x0 = e._e(M, D)
    x0b = e._e(M, D, dtype=BF16)
    seed_ln = _site_seed(base_seed, 8)
    st_enc = e._ln(xe, "audio_encoder.encoder.layer_norm", c.layer_norm_eps, y=x0, yb=x0b, drop_p=hp, seed=seed_ln)
    ctx.update(a_b=B, a_T=T, a_maskf=maskf, a_mask32=mask32, a_spec=spec,
               w2v=dict(wave=wave, N=N, Ts=Ts, y0=y0, gn_mean=gn_mean, gn_rstd=gn_rstd, convs=convs, a0=a0, st0=st0,
                        conv_out=h, p_fp=p_fp, seed_fp=seed_fp, norms=norms, wf=wf, xp=xp, cpad=cpad, xe=xe,
                        st_enc=st_enc, seed_ln=seed_ln, hp=hp, ap=ap, act_p=act_p))
    if not save:
        ctx["w2v"] = None
    # ---- post-LN layers (layerdrop as transformers :700-712)
    layers = []
    x, xb = x0, x0b
    for i in range(c.num_hidden_layers):
        if train and c.layerdrop > 0 and float(torch.rand([], generator=e.layerdrop_gen)) < c.layerdrop:
            layers.append(None)
            continue
        x, xb, sv = e._postln_fwd(c, W2V2_NAMES, i, x, xb, B, T, mask32, hp, ap, _site_seed(base_seed, 100 + i),
                                  save, act_p=act_p)
        layers.append(sv if save else None)
    ctx["a_layers"] = layers
    return x, xb


def _pos_gemm(xp, w, out, rows, G, Cg, Kp, seg):
    """out[:, g·Cg:(g+1)·Cg] = im2col(xp[g]) · w[g]ᵀ for every group g in one batched GEMM: the
    im2col row r is xp[g][r : r + Kp] (Kp·Cg contiguous elements), i.e. a view with row stride Cg."""
    a = torch.as_strided(xp, (rows, Kp * Cg), (Cg, 1))
    b = w.view(G * Cg, Kp * Cg)[:Cg]
    D = G * Cg
    o = torch.as_strided(out, (rows, Cg), (D, 1))
    ops.gemm(a, b, M=rows, N=Cg, K=Kp * Cg, batch=G, stride_a=seg * Cg, stride_b=Cg * Kp * Cg, stride_c=Cg, out=o)


def backward(e, dh, ctx, layers_done=None):
    """dh fp32 [B*T, D] (d last_hidden_state) -> parameter gradients of the wav2vec2 encoder."""
    from .engine import W2V2_NAMES
    c = e.acfg
    s = e.s
    sv = ctx["w2v"]
    B, T = ctx["a_b"], ctx["a_T"]
    maskf, mask32 = ctx["a_maskf"], ctx["a_mask32"]
    D = c.hidden_size
    M = B * T
    lo = next((i for i in range(c.num_hidden_layers)
               if s.trainable_layer(f"audio_encoder.encoder.layers.{i}.attention.q_proj.weight")), None)
    dx = dh
    for i in reversed(range(c.num_hidden_layers)):
        lsv = ctx["a_layers"][i]
        if lsv is not None:
            dx = e._postln_bwd(c, W2V2_NAMES, i, lsv, dx, B, T, mask32, sv["hp"], sv["ap"])
            ctx["a_layers"][i] = None
        if layers_done is not None and i == lo:
            layers_done()
    if lo is None and layers_done is not None:
        layers_done()
    if not _needs_grad_below_layers(s):
        return
    # ---- encoder LayerNorm (its output dropout undone on dy)
    dxe = e._e(M, D)
    e._ln_bwd(dx, sv["xe"], sv["st_enc"], "audio_encoder.encoder.layer_norm", dx=dxe, in_drop_p=sv["hp"],
              in_seed=sv["seed_ln"])
    # ---- positional conv: xe = x + gelu(conv(x) + bias)
    G, Kp = c.num_conv_pos_embedding_groups, c.num_conv_pos_embeddings
    Cg = D // G
    Tp = T + Kp - 1
    seg = B * Tp + Kp
    bias = s.p(PC + "bias")
    dpc = e._e(M, D)
    _lib.call("ste_w2v_pos_elem", 1, ptr(sv["cpad"]), ptr(bias), ptr(dxe), None, B, T, D, Tp, ptr(dpc), _s())
    gb = s.g(PC + "bias")
    if gb is not None:
        ops.colsum(dpc, gb)
    dyp = e._e(G * seg * Cg, dtype=BF16)
    _lib.call("ste_w2v_pos_pack", ptr(dpc), B, T, D, G, Kp, Kp - 1 - Kp // 2, ptr(dyp), _s())
    del dpc
    gv, gg = s.g(PC + "parametrizations.weight.original1"), s.g(PC + "parametrizations.weight.original0")
    if gv is not None or gg is not None:
        # dW_g[co, (j, ci)] = Σ_rows dY[row, co] · xp_g[row + j, ci]; the padded dY copy is shifted
        # by Kp-1-Kp//2 rows relative to xp, which the A pointer offset undoes
        shift = (Kp - 1 - Kp // 2) * Cg
        a = torch.as_strided(dyp, (B * Tp, Cg), (Cg, 1), shift)
        b = torch.as_strided(sv["xp"], (B * Tp, Kp * Cg), (Cg, 1))
        dwr = e._e(G * Cg, Kp * Cg)
        ops.gemm(a, b, a_kc=False, b_kc=False, M=Cg, N=Kp * Cg, K=B * Tp, batch=G, stride_a=seg * Cg,
                 stride_b=seg * Cg, stride_c=Cg * Kp * Cg, out=dwr)
        _lib.call("ste_w2v_wnorm_bwd", ptr(dwr), ptr(s.p(PC + "parametrizations.weight.original1")),
                  ptr(s.p(PC + "parametrizations.weight.original0")), ptr(sv["norms"]), D, Cg, Kp, ptr(gv), ptr(gg),
                  _s())
        del dwr
    dxpad = e._e(B * Tp, D)
    _pos_gemm(dyp, sv["wf"], dxpad, B * Tp, G, Cg, Kp, seg)
    del dyp
    dx = e._e(M, D)
    _lib.call("ste_w2v_pos_elem", 2, ptr(dxpad), None, ptr(dxe), ptr(maskf), B, T, D, Tp, ptr(dx), _s())
    del dxpad, dxe
    # ---- SpecAugment rows, dropout + frame mask of the projection output
    if ctx.get("a_spec") is not None:
        ops.spec_mask_bwd(dx, ctx["a_spec"], maskf, s.g("audio_encoder.masked_spec_embed"))
    _lib.call("ste_w2v_drop_rows", ptr(dx), M, D, float(sv["p_fp"]), int(sv["seed_fp"]) & (2**64 - 1), ptr(maskf),
              _s())
    # ---- feature projection
    dxb = ops.cast_bf16(dx, e._e(M, D, dtype=BF16))
    e._dw(dxb, sv["a0"], "audio_encoder.feature_projection.projection.weight")
    e._db(dxb, "audio_encoder.feature_projection.projection.bias")
    if not _needs_grad_conv(s, c):
        return
    da0 = ops.linear_dx(dxb, s.w("audio_encoder.feature_projection.projection.weight"))
    del dxb
    Ts = sv["Ts"]
    nl = len(c.conv_dim)
    dcur = e._e(B * Ts[nl], c.conv_dim[-1])
    e._ln_bwd(da0, sv["conv_out"], sv["st0"], "audio_encoder.feature_projection.layer_norm", dx=dcur)
    del da0
    # ---- conv stack, top down: dz_l = dh_l · gelu'(z_l) (bf16), dW_l, dcol -> fold -> dh_{l-1}
    convs = sv["convs"]
    cl = c.conv_dim[-1]
    dz = e._e(B * Ts[nl], cl, dtype=BF16)
    _lib.call("ste_w2v_conv_fold", ptr(dcur), cl, ptr(convs[nl - 1]["z"]), B, Ts[nl], Ts[nl], cl, 1, 1, ptr(dz), 1,
              _s())
    del dcur
    for l in range(nl - 1, 0, -1):
        cin, cout, k, st = c.conv_dim[l - 1], c.conv_dim[l], c.conv_kernel[l], c.conv_stride[l]
        Ti, To = Ts[l], Ts[l + 1]
        hin = convs[l - 1]["h"]
        gw = s.g(FE + f"{l}.conv.weight")
        if gw is not None:
            # per-clip dW slabs [B][Co][k·Ci] (the strided views of different clips are not one
            # uniform k-major matrix), summed in fixed order, then permuted into [Co][Ci][k]
            part = e._e(B * cout, k * cin)
            b = torch.as_strided(hin, (To, k * cin), (st * cin, 1))
            ops.gemm(dz, b, a_kc=False, b_kc=False, M=cout, N=k * cin, K=To, batch=B, stride_a=To * cout,
                     stride_b=Ti * cin, stride_c=cout * k * cin, out=part)
            dwr = e._z(cout, k * cin)
            _lib.call("ste_w2v_slab_sum", ptr(dwr), ptr(part), cout * k * cin, B, _s())
            del part
            _lib.call("ste_w2v_perm12", ptr(dwr), ptr(gw), cout, k, cin, 1, _s())
            del dwr
        if l == 1 and not _needs_grad_conv0(s):
            break
        dcol = ops.linear_dx(dz, convs[l]["wr"])          # [B*To, k·Ci] fp32
        first = l == 1
        dprev = e._e(B * Ti, cin, dtype=F32 if first else BF16)
        _lib.call("ste_w2v_conv_fold", ptr(dcol), k * cin, None if first else ptr(convs[l - 1]["z"]), B, Ti, To, cin,
                  k, st, ptr(dprev), 0 if first else 1, _s())
        del dcol
        dz = dprev
    else:
        # ---- conv0 + GroupNorm + GELU (dz is dL/dh0 in fp32 here)
        C0, K0, S0 = c.conv_dim[0], c.conv_kernel[0], c.conv_stride[0]
        T0 = Ts[1]
        nwork = int(_lib.fn("ste_w2v_gn_work")(B, T0, C0, K0))
        work = e._e(nwork)
        _lib.call("ste_w2v_gn_bwd", ptr(dz), ptr(sv["y0"]), ptr(sv["gn_mean"]), ptr(sv["gn_rstd"]),
                  ptr(s.p(FE + "0.layer_norm.weight")), ptr(s.p(FE + "0.layer_norm.bias")), ptr(sv["wave"]),
                  sv["wave"].stride(0), B, sv["N"], T0, C0, K0, S0, ptr(s.g(FE + "0.layer_norm.weight")),
                  ptr(s.g(FE + "0.layer_norm.bias")), ptr(s.g(FE + "0.conv.weight")), ptr(work), nwork, _s())


def _needs_grad_conv0(s):
    return any(s.g(FE + n) is not None for n in ("0.conv.weight", "0.layer_norm.weight", "0.layer_norm.bias"))


def _needs_grad_conv(s, c):
    return any(s.g(FE + f"{l}.conv.weight") is not None for l in range(len(c.conv_dim))) or _needs_grad_conv0(s)


def _needs_grad_below_layers(s):
    names = ["audio_encoder.encoder.layer_norm.weight", PC + "bias", PC + "parametrizations.weight.original1",
             "audio_encoder.feature_projection.projection.weight", "audio_encoder.masked_spec_embed",
             FE + "0.conv.weight"]
    return any(n in s.slots and s.g(n) is not None for n in names)
