"""Precision probe of the audio encoder's gradients — test tooling, imports oracle/.

Question: the HIP path's full-size per-tensor gradient errors against the fp32 oracle peak at
1.75-2.06 % on the trainable Conformer layers' linear_q/k, distance_embedding and the audio
pooling scorer (profiles/r3_parity.txt).  Is that the bf16 floor of the reference graph itself,
and which rounding point carries it?

Method (CPU, no GPU): the w2v-bert-2.0 Conformer (24 x 1024, full c2 shapes: B = 2 clips of
10 s = 499 frames, 3 trainable layers + the feature projection, eval mode) and the audio
attentive pooling, with a fixed random cotangent on the pooled output, run
  * in fp32 (the oracle's math, oracle/ref_model.py:84-150, 197-203), and
  * with bf16 rounding injected at the points the HIP path rounds (engine._conformer_fwd/_bwd,
    csrc/attention.hip attn_bwd_*_rel3), each point behind a flag:
      w    GEMM weight operands and the distance table E in bf16 (ParamStore's shadow)
      fa   forward activations stored bf16: every GEMM's A operand (LayerNorm yb outputs, the
           swish outputs, O), the q/k/v, pw1 and depthwise-conv outputs
      bdy  backward GEMM dY operands in bf16 (dx·0.5 / dx / dqkv as the dX and dW GEMMs read them)
      bdx  backward dX GEMM outputs in bf16 (the out_bf16 input gradients feeding LayerNorm and
           attention backwards)
      ads  attention dS and its distance-bin sums G rounded to bf16 for dQ = dS·K + G·E and
           dK = dSᵀ·Q (pack_acc in attn_bwd_dq_rel3 / dkv_rel3)
      apb  attention P rounded to bf16 for dV = Pᵀ·dO
      zb   the FFN swish's pre-activation z stored bf16 for the backward (the FFN-in GEMM's
           pre_out copy that the activation-backward epilogue reads: swish'(bf16(z)); round 5)
    (the forward's P·V runs on P = hi + lo, ~fp32, as the saving forward does; the pooling
    scorer reads the fp32 states — the [hi | lo] split image — with bf16 W.)
Per-tensor gradient error = ||g - g_fp32|| / ||g_fp32||, printed for every flag set: all on
(the HIP path's rounding), all off, the reference graph under bf16 autocast (scores and
probabilities in bf16 storage as CUDA autocast leaves them), and all-on-minus-one.

    python tests/precision_probe.py [--layers 24] [--threads 8] [--sets all,hip,...]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import fbank_ref, ref_model as R  # noqa: E402

FLAGS = ("w", "fa", "bdy", "bdx", "ads", "apb", "zb")
# weight classes for the "w" attribution sets (w_<class>): which GEMMs read bf16 weights
WCLASSES = ("qkv", "E", "o", "ffn", "conv", "pool", "fp")


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


class _Q(torch.autograd.Function):
    """Round to bf16 in the forward (f) and/or the incoming gradient in the backward (b)."""

    @staticmethod
    def forward(ctx, x, f, b):
        ctx.b = b
        return bf(x) if f else x.clone()

    @staticmethod
    def backward(ctx, g):
        return (bf(g) if ctx.b else g), None, None


class _SiluZ(torch.autograd.Function):
    """swish whose backward reads the pre-activation from a bf16 copy (zb)."""

    @staticmethod
    def forward(ctx, z):
        ctx.save_for_backward(bf(z))
        return F.silu(z)

    @staticmethod
    def backward(ctx, g):
        z, = ctx.saved_tensors
        sg = torch.sigmoid(z)
        return g * sg * (1 + z * (1 - sg))


def q(x, f, b):
    return _Q.apply(x, bool(f), bool(b)) if (f or b) else x


def mx8(x):
    """OCP MX-fp8 round trip along the last dim (ste_mx8_quant): blocks of 32, scale
    2^ceil(log2(amax / 448)) (no saturation), e4m3 round-to-nearest-even, dequantised."""
    shp = x.shape
    xb = x.reshape(-1, shp[-1] // 32, 32)
    amax = xb.abs().amax(-1, keepdim=True)
    e = torch.ceil(torch.log2(torch.clamp(amax, min=1e-30) / 448.0))
    scale = torch.where(amax > 0, torch.exp2(e), torch.full_like(amax, 2.0 ** -127))
    qv = (xb / scale).to(torch.float8_e4m3fn).to(torch.float32)
    return (qv * scale).reshape(shp)


class _LinMX8(torch.autograd.Function):
    """config 5's fp8 forward GEMM: y = mx8(x)·mx8(W)ᵀ + b; straight-through backward on the bf16
    operands (dX = dY·W, dW = dYᵀ·x), as engine.py's fp8_gemm path runs it."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return F.linear(mx8(x), mx8(W), b)

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        gx = g @ W
        gW = g.reshape(-1, g.shape[-1]).t() @ x.reshape(-1, x.shape[-1])
        gb = g.reshape(-1, g.shape[-1]).sum(0) if ctx.has_b else None
        return gx, gW, gb


class Probe:
    def __init__(self, fl, autocast=False, wclasses=WCLASSES, wlayers=None, fasites=None, falayers=None,
                 fp8=(), olo=None, plo=False):
        self.fl = {k: bool(fl.get(k, False)) for k in FLAGS}
        self.ac = autocast   # reference-under-autocast: scores / probabilities in bf16 storage too
        self.wclasses = set(wclasses)
        self.wlayers = wlayers   # None: every layer's weights bf16 (with "w"); else a set of layer indices
        self.layer = None
        self.fasites = None if fasites is None else set(fasites)   # None: every site rounds (with "fa")
        self.falayers = falayers
        self.fp8 = set(fp8)   # GEMM classes (qkv, o, ffn, conv) on MX-fp8 forward operands (config 5)
        # diagnostics of the attention's own approximations (not bf16 storage): olo = how the
        # backward's delta = dO·O reads O ("bf16": hi + bf16 lo, the ste_attn_args.o_lo image;
        # "fp16s": hi + fp16 lo scaled by 2^8; None: fp32); plo: the forward's PV on P = hi + lo
        # (True: normalised by the fp32 Σ p, as attn_fwd_rel4<*, true> through round 5; "norm": by
        # the Σ of the same hi + lo P)
        self.olo = olo
        self.plo = plo

    def fa(self, site):
        """forward rounding of an activation at `site` (qkv_in, qkv_out, o, ffn_in, ffn_h, conv_in,
        pw1, cv, sw, fp_in)"""
        if not self.fl["fa"]:
            return False
        if self.fasites is not None and site not in self.fasites:
            return False
        return self.falayers is None or self.layer is None or self.layer in self.falayers

    def wq(self, W, cls):
        on = self.fl["w"] and cls in self.wclasses and (self.wlayers is None or self.layer is None or
                                                       self.layer in self.wlayers)
        return q(W, on, False)

    def lin(self, x, W, b=None, out_site=None, dx_round=True, in_site="ffn_in", cls="ffn"):
        """nn.Linear as ste_gemm: A operand bf16 (fa at in_site, and its gradient bf16 if dx_round
        & bdx), B operand bf16 (w), fp32 accumulation, output bf16 storage (fa at out_site) and the
        dY operand of the backward GEMMs bf16 (bdy)."""
        fl = self.fl
        xa = q(x, self.fa(in_site), fl["bdx"] and dx_round)
        Wa = self.wq(W, cls)
        y = _LinMX8.apply(xa, Wa, b) if (cls in self.fp8 and self.layer is not None) else F.linear(xa, Wa, b)
        return q(y, out_site is not None and self.fa(out_site), fl["bdy"])

    def ln(self, p, name, x, eps=1e-5):
        return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)

    # ------------------------------------------------------------------ Conformer pieces
    def ffn(self, p, pre, a):
        z = self.lin(a, p[pre + "intermediate_dense.weight"], p[pre + "intermediate_dense.bias"])
        sw = _SiluZ.apply(z) if self.fl["zb"] else F.silu(z)
        h = q(sw, self.fa("ffn_h"), False)     # swish epilogue, stored bf16; dz rounded by the GEMM's bdy
        return self.lin(h, p[pre + "output_dense.weight"], p[pre + "output_dense.bias"], dx_round=False,
                        in_site="ffn_h")

    def attn(self, p, pre, a, cfg):
        B, T, D = a.shape
        H, d = cfg.heads, D // cfg.heads
        W = torch.cat([p[pre + "linear_q.weight"], p[pre + "linear_k.weight"], p[pre + "linear_v.weight"]], 0)
        bq = torch.cat([p[pre + "linear_q.bias"], p[pre + "linear_k.bias"], p[pre + "linear_v.bias"]], 0)
        qkv = self.lin(a, W, bq, out_site="qkv_out", in_site="qkv_in", cls="qkv")
        qh, kh, vh = (t.reshape(B, T, H, d).transpose(1, 2) for t in qkv.split(D, -1))
        E = self.wq(p[pre + "distance_embedding.weight"], "E")
        o = _Attn.apply(qh, kh, vh, E, 1.0 / math.sqrt(d), cfg.left, cfg.right, self)
        o = o.transpose(1, 2).reshape(B, T, D)
        return self.lin(o, p[pre + "linear_out.weight"], p[pre + "linear_out.bias"], in_site="o", cls="o")

    def conv(self, p, pre, x2, cfg):
        a = self.ln(p, pre + "layer_norm", x2, cfg.eps)
        D = a.shape[-1]
        pw1 = self.lin(a, p[pre + "pointwise_conv1.weight"].view(2 * D, D), None, out_site="pw1", in_site="conv_in",
                       cls="conv")
        g = F.glu(pw1, dim=-1).transpose(1, 2)
        g = F.pad(g, (cfg.conv_k - 1, 0))
        cv = F.conv1d(g, p[pre + "depthwise_conv.weight"], groups=D).transpose(1, 2)
        cv = q(cv, self.fa("cv"), self.fl["bdx"])          # cv bf16; its gradient (dcv) bf16
        sw = F.silu(self.ln(p, pre + "depthwise_layer_norm", cv, cfg.eps))
        return self.lin(sw, p[pre + "pointwise_conv2.weight"].view(D, D), None, in_site="sw", cls="conv")

    def encoder(self, p, feats, cfg, layers):
        x = self.ln(p, "audio_encoder.feature_projection.layer_norm", feats, cfg.eps)
        h = self.lin(x, p["audio_encoder.feature_projection.projection.weight"],
                     p["audio_encoder.feature_projection.projection.bias"], in_site="fp_in", cls="fp")
        for i in range(cfg.layers - layers, cfg.layers):
            self.layer = i
            pre = f"audio_encoder.encoder.layers.{i}."
            h = h + 0.5 * self.ffn(p, pre + "ffn1.", self.ln(p, pre + "ffn1_layer_norm", h, cfg.eps))
            h = h + self.attn(p, pre + "self_attn.", self.ln(p, pre + "self_attn_layer_norm", h, cfg.eps), cfg)
            h = h + self.conv(p, pre + "conv_module.", h, cfg)
            h = h + 0.5 * self.ffn(p, pre + "ffn2.", self.ln(p, pre + "ffn2_layer_norm", h, cfg.eps))
            h = self.ln(p, pre + "final_layer_norm", h, cfg.eps)
        self.layer = None
        return h

    def pool(self, p, h):
        """AttentivePooling as the HIP path runs it: fp32 states (split image), bf16 W1, fp32 rest."""
        W1 = self.wq(p["audio_pooling.attention.0.weight"], "pool")
        t = torch.tanh(F.linear(h, W1, p["audio_pooling.attention.0.bias"]))
        s = F.linear(t, p["audio_pooling.attention.2.weight"], p["audio_pooling.attention.2.bias"]).squeeze(-1)
        w = torch.softmax(s, dim=1)
        return torch.bmm(w.unsqueeze(1), h).squeeze(1)


class _Attn(torch.autograd.Function):
    """Relative-key attention (w2v:229-327) with the HIP kernels' rounding points."""

    @staticmethod
    def forward(ctx, qh, kh, vh, E, scale, left, right, pr):
        B, H, T, d = qh.shape
        pos = torch.arange(T)
        dist = ((pos.view(1, -1) - pos.view(-1, 1)).clamp(-left, right) + left)
        s = qh @ kh.transpose(-1, -2)
        qe = qh @ E.t()
        s = (s + torch.gather(qe, 3, dist.view(1, 1, T, T).expand(B, H, T, T))) * scale
        if pr.ac:
            s = bf(s)
        p = torch.softmax(s, -1)
        if pr.plo:
            ph = bf(p)
            pp = ph + bf(p - ph)
            o = pp @ vh
            if pr.plo == "norm":   # O's weights renormalised to sum to 1 (Σ of the same hi + lo P)
                o = o / pp.sum(-1, keepdim=True)
        else:
            o = (bf(p) if pr.ac else p) @ vh
        if pr.ac:
            o = bf(o)
        ctx.save_for_backward(qh, kh, vh, E, p, o)
        ctx.dist, ctx.scale, ctx.pr = dist, scale, pr
        return o

    @staticmethod
    def backward(ctx, do):
        qh, kh, vh, E, p, o = ctx.saved_tensors
        fl, ac = ctx.pr.fl, ctx.pr.ac
        B, H, T, d = qh.shape
        nrel = E.shape[0]
        dp = do @ vh.transpose(-1, -2)
        od = o
        if ctx.pr.olo is not None:
            oh = bf(o)
            od = oh + (bf(o - oh) if ctx.pr.olo == "bf16" else
                       ((o - oh) * 256.0).to(torch.float16).to(torch.float32) / 256.0)
        delta = (do * od).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        if ac:
            ds = bf(ds)
        G = torch.zeros(B, H, T, nrel).scatter_add_(3, ctx.dist.view(1, 1, T, T).expand(B, H, T, T), ds)
        dsr = bf(ds) if fl["ads"] else ds
        Gr = bf(G) if fl["ads"] else G
        dq = (dsr @ kh + Gr @ E) * ctx.scale
        dk = (dsr.transpose(-1, -2) @ qh) * ctx.scale
        pb = bf(p) if (fl["apb"] or ac) else p
        dv = pb.transpose(-1, -2) @ do
        dE = (G.transpose(-1, -2) @ qh).sum((0, 1)) * ctx.scale
        return dq, dk, dv, dE, None, None, None, None


def init_params(cfg, seed=0):
    """The GPU model's init rule (model.py _init_params): encoder weights N(0, 0.02), LayerNorms
    1/0, encoder biases 0, heads as nn.Linear defaults."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for n, shp in R.param_shapes(cfg, spec_augment=False):
        if not (n.startswith("audio_encoder") or n.startswith("audio_pooling")):
            continue
        leaf = n.rsplit(".", 1)[-1]
        if ("norm" in n.lower()) and leaf in ("weight", "bias"):
            t = torch.ones(shp) if leaf == "weight" else torch.zeros(shp)
        elif n.startswith("audio_encoder"):
            t = torch.zeros(shp) if leaf == "bias" else torch.randn(shp, generator=g) * 0.02
        else:
            fan_in = shp[-1] if len(shp) > 1 else shp[0]
            t = (torch.rand(shp, generator=g) * 2 - 1) * fan_in ** -0.5
        p[n] = t
    return p


def run(p0, feats, cot, cfg, layers, trainable, fl, autocast=False, round_feats=False, **kw):
    pr = Probe(fl, autocast, **kw)
    if round_feats:
        feats = bf(feats)
    p = {n: t.clone().requires_grad_(n in trainable) for n, t in p0.items()}
    h = pr.encoder(p, feats, cfg, layers)
    pooled = pr.pool(p, h)
    pooled.backward(cot)
    return {n: p[n].grad.clone() for n in trainable if p[n].grad is not None}, pooled.detach()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--unfreeze", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--sets", default="hip,autocast,minus")
    ap.add_argument("--json", default=None)
    ap.add_argument("--seed", type=int, default=0, help="weights / clips / cotangent draw (instance variance)")
    args = ap.parse_args(argv)
    torch.set_num_threads(args.threads)
    cfg = R.ModelCfg()
    ac = cfg.audio
    p0 = init_params(cfg, args.seed)
    n = int(args.seconds * 16000)
    feats, _ = fbank_ref.collate([fbank_ref.extract(fbank_ref.synth_wave(1000 + 100 * args.seed + i, n))[0]
                                  for i in range(args.batch)])
    feats = torch.as_tensor(np.asarray(feats), dtype=torch.float32)
    top = [f"audio_encoder.encoder.layers.{i}." for i in range(ac.layers - args.unfreeze, ac.layers)]
    trainable = {k for k in p0 if k.startswith("audio_encoder.feature_projection") or k.startswith("audio_pooling")
                 or any(k.startswith(t) for t in top)}
    cot = torch.randn(args.batch, ac.hidden, generator=torch.Generator().manual_seed(5 + args.seed))
    t0 = time.time()
    ref, out_ref = run(p0, feats, cot, ac, args.layers, trainable, {})
    print(f"fp32 reference: {time.time() - t0:.1f} s, {len(ref)} gradient tensors", flush=True)
    sets = []
    want = args.sets.split(",")
    allon = {k: True for k in FLAGS}
    if "hip" in want:
        sets.append(("hip (all flags)", allon, False))
    if "autocast" in want:
        sets.append(("reference under bf16 autocast", {"w": True, "fa": True, "bdy": True, "bdx": True, "ads": True,
                                                       "apb": True}, True))
    if "minus" in want:
        sets += [(f"hip minus {k}", {**allon, k: False}, False) for k in FLAGS]
    for k in FLAGS:
        if f"only_{k}" in want:
            sets.append((f"only {k}", {k: True}, False))
    if "now" in want:
        sets.append(("hip, bf16-exact weights", {**allon, "w": False}, False))
    if "nowminus" in want:   # bf16-representable weights (no weight rounding), then one more point off
        now = {**allon, "w": False}
        sets.append(("hip, bf16-exact weights", now, False))
        sets += [(f"hip, bf16-exact weights, minus {k}", {**now, k: False}, False) for k in FLAGS if k != "w"]
    FASITES = ("qkv_in", "qkv_out", "o", "ffn_in", "ffn_h", "conv_in", "pw1", "cv", "sw", "fp_in")
    if "fasite" in want:   # bf16-exact weights, forward rounding at one site only
        now = {**allon, "w": False}
        sets += [(f"hip, bf16-exact weights, fwd rounding only at {st}", now, False, dict(fasites=(st,)))
                 for st in FASITES]
    if "falayers" in want:
        now = {**allon, "w": False}
        topl = set(range(ac.layers - args.unfreeze, ac.layers))
        sets += [("hip, bf16-exact weights, fwd rounding only in the trainable layers", now, False,
                  dict(falayers=topl)),
                 ("hip, bf16-exact weights, fwd rounding only in the frozen layers", now, False,
                  dict(falayers=set(range(ac.layers)) - topl))]
    if "wclass" in want:   # everything else on, bf16 weights in one class only
        sets += [(f"hip, bf16 weights only in {c}", allon, False, dict(wclasses=(c,))) for c in WCLASSES]
    if "wlayers" in want:  # bf16 weights only in the trainable / frozen layers
        topl = set(range(ac.layers - args.unfreeze, ac.layers))
        sets += [("hip, bf16 weights only in the trainable layers", allon, False, dict(wlayers=topl)),
                 ("hip, bf16 weights only in the frozen layers", allon, False,
                  dict(wlayers=set(range(ac.layers)) - topl))]
    if "fp8" in want:   # config 5: MX-fp8 forward GEMMs of the Conformer layers, by GEMM class
        allc = ("qkv", "o", "ffn", "conv")
        sets.append(("hip + fp8 forward GEMMs (all classes)", allon, False, dict(fp8=allc)))
        sets += [(f"hip + fp8 forward GEMMs except {c}", allon, False, dict(fp8=tuple(x for x in allc if x != c)))
                 for c in allc]
        sets += [(f"hip + fp8 forward GEMMs only {c}", allon, False, dict(fp8=(c,))) for c in allc]
    if "inputs" in want:   # conditioning: the fp32 graph on input features rounded to bf16 (one ulp)
        sets.append(("fp32 graph, input features rounded to bf16", {}, False, dict(round_feats=True)))
        sets.append(("fp32 graph, weights rounded to bf16", {"w": True}, False))
    results = {}
    for item in sets:
        name, fl, acm = item[:3]
        kw = item[3] if len(item) > 3 else {}
        t0 = time.time()
        g, out = run(p0, feats, cot, ac, args.layers, trainable, fl, acm, **kw)
        errs = sorted(((((g[k] - ref[k]).norm() / ref[k].norm()).item(), k) for k in ref
                       if ref[k].norm() > 1e-8 and not k.endswith(("linear_k.bias", "attention.2.bias"))), reverse=True)
        med = errs[len(errs) // 2][0]
        oerr = ((out - out_ref).norm() / out_ref.norm()).item()
        results[name] = {"worst": errs[:6], "median": med, "pooled_err": oerr}
        print(f"[{name}] {time.time() - t0:.0f}s pooled {oerr:.2e} median {med:.2e} worst "
              + ", ".join(f"{e:.4f} {k.replace('audio_encoder.encoder.', '')}" for e, k in errs[:5]), flush=True)
    if args.json:
        Path(args.json).write_text(json.dumps(results, indent=1))


if __name__ == "__main__":
    main()
