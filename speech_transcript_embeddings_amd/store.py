r"""Flat parameter storage in HBM.

Every parameter of the model tree becomes a view into ONE fp32 master buffer;
trainable parameters that receive gradients come first, so their gradients,
Adam moments and the fused optimizer work on contiguous ranges:

  [ encoder params with grad | head params with grad | trainable-without-grad | frozen ]
    \_____ grad / exp_avg / exp_avg_sq cover this prefix ____/

The encoder / head split mirrors the reference's two AdamW param groups
(ref:training/trainer_unfreeze.py:1496-1511: names containing 'text_encoder' or
'audio_encoder' get lr/50).  Parameters the reference never gives a gradient
(text pooler, masked_spec_embed without SpecAugment: grad None -> AdamW skips them)
sit in the third segment.

A bf16 shadow with the same offsets holds the MFMA operands.  The fused optimizer
refreshes it for updated ranges; anything else that writes parameters (load_state_dict,
a torch optimizer) bumps the tensor version counter and the shadow is re-cast lazily.

Fused groups (q/k/v weights and biases, key/value of the cross-modal attentions) are
laid out adjacently so one GEMM serves them and one dW GEMM writes their gradients.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import ops

ALIGN = 8  # elements: 32 B for fp32, 16 B for the bf16 shadow


def _fuse_groups(names):
    """Return name -> tuple(group) for parameters that must be adjacent."""
    groups = {}
    sets = [("attention.self.query", "attention.self.key", "attention.self.value"),
            ("self_attn.linear_q", "self_attn.linear_k", "self_attn.linear_v"),
            ("attention.q_proj", "attention.k_proj", "attention.v_proj"),
            ("_attention.key", "_attention.value")]
    nameset = set(names)
    for n in names:
        for trio in sets:
            for leaf in ("weight", "bias"):
                head = trio[0] + "." + leaf
                if n.endswith(head):
                    prefix = n[: -len(head)]
                    grp = tuple(prefix + t + "." + leaf for t in trio)
                    if all(g in nameset for g in grp):
                        for g in grp:
                            groups[g] = grp
    return groups


@dataclass
class Slot:
    name: str
    offset: int
    numel: int
    shape: tuple
    segment: str


class ParamStore:
    def __init__(self, model: torch.nn.Module, device, has_grad: set[str]):
        named = list(model.named_parameters())
        names = [n for n, _ in named]
        params = dict(named)
        groups = _fuse_groups(names)

        def seg_of(n, p):
            if not p.requires_grad:
                return "frozen"
            if n not in has_grad:
                return "nograd"
            return "enc" if ("text_encoder" in n or "audio_encoder" in n) else "head"

        order = {"enc": [], "head": [], "nograd": [], "frozen": []}
        seen = set()
        for n, p in named:
            if n in seen:
                continue
            grp = groups.get(n, (n,))
            segs = {seg_of(g, params[g]) for g in grp}
            if len(segs) != 1:
                grp = (n,)
            for g in grp:
                order[seg_of(g, params[g])].append(g)
                seen.add(g)
        self.slots: dict[str, Slot] = {}
        off = 0
        self.seg_range = {}
        for seg in ("enc", "head", "nograd", "frozen"):
            start = off
            for n in order[seg]:
                p = params[n]
                grp = groups.get(n)
                if grp is None or n == grp[0]:
                    off = (off + ALIGN - 1) // ALIGN * ALIGN
                self.slots[n] = Slot(n, off, p.numel(), tuple(p.shape), seg)
                off += p.numel()
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            self.seg_range[seg] = (start, off)
        self.numel = off
        self.n_grad = self.seg_range["head"][1]
        self.device = torch.device(device)
        self.master = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        self.shadow = torch.zeros(self.numel, device=self.device, dtype=torch.bfloat16)
        self.grad = torch.zeros(self.n_grad, device=self.device, dtype=torch.float32)
        # re-seat every parameter as a view of the flat buffer (module trees may be built on
        # the meta device: values are initialised afterwards, directly in HBM)
        for n, s in self.slots.items():
            p = params[n]
            view = self.master[s.offset:s.offset + s.numel].view(s.shape)
            if p.device.type != "meta":
                with torch.no_grad():
                    view.copy_(p.detach().to(self.device, torch.float32))
            owner, leaf = (model.get_submodule(n.rsplit(".", 1)[0]), n.rsplit(".", 1)[1]) if "." in n \
                else (model, n)
            newp = torch.nn.Parameter(view, requires_grad=p.requires_grad)
            owner._parameters[leaf] = newp
            params[n] = newp
        self.params = params
        self._versions = {}
        self._wt = {}          # (name, count) -> (Wᵀ bf16, param versions, opt_epoch) (see wt())
        self._wq = {}          # (name, count) -> ((W e4m3, E8M0 scales), versions, opt_epoch) (see wq())
        self._wtq = {}         # (name, count) -> ((Wᵀ e4m3, E8M0 scales), the wt() tensor, its rebuild stamp)
        self._w2 = {}          # (name, count) -> ([W | W] bf16 [out, 2·in], versions, opt_epoch) (see w2())
        self._wt2 = {}         # (name, count) -> ([Wᵀ | Wᵀ], the wt() tensor, its rebuild stamp) (see wt2())
        self._wt_stamp = {}    # (name, count) -> number of wt() rebuilds (wt2 follows them)
        self.opt_epoch = 0     # fused optimizer steps so far (each refreshes the shadow of every trained weight)
        self._prebuilt = None  # (event, stream, streams that waited): Wᵀ rebuilt by refresh_transposes
        self.sync_shadow(force=True)

    # ------------------------------------------------------------------ views
    def p(self, name):
        s = self.slots[name]
        return self.master[s.offset:s.offset + s.numel].view(s.shape)

    def w(self, name, rows=None):
        """bf16 shadow as a 2-D [out, in] matrix (conv weights [out,in,1] flattened)."""
        s = self.slots[name]
        v = self.shadow[s.offset:s.offset + s.numel]
        return v.view(s.shape[0], -1) if rows is None else v.view(rows, -1)

    def g(self, name):
        s = self.slots[name]
        if s.segment not in ("enc", "head"):
            return None
        return self.grad[s.offset:s.offset + s.numel].view(s.shape)

    def fused(self, first: str, count: int, which: str):
        """Adjacent group starting at `first` as one tensor: which in {'w','p','g'}."""
        s = self.slots[first]
        n = s.numel * count
        if which == "w":
            return self.shadow[s.offset:s.offset + n].view(s.shape[0] * count, -1)
        if which == "p":
            base = self.master[s.offset:s.offset + n]
            return base.view(s.shape[0] * count, *s.shape[1:]) if len(s.shape) > 1 else base
        if s.segment not in ("enc", "head"):
            return None
        base = self.grad[s.offset:s.offset + n]
        return base.view(s.shape[0] * count, *s.shape[1:]) if len(s.shape) > 1 else base

    def _group_versions(self, name, count):
        s = self.slots[name]
        if count == 1:
            names = [name]
        else:
            names = [n for n, t in self.slots.items() if s.offset <= t.offset < s.offset + s.numel * count]
        return tuple(self.params[n]._version for n in names), s.segment in ("enc", "head")

    def wq(self, name: str, count: int = 1):
        """W as MX-fp8 (e4m3 [out, in] + E8M0 scales [out, in/32]), the B operand of the MX-fp8
        forward GEMMs (model fp8_gemm=True, BASELINE config 5).  Quantised from the bf16 shadow
        and cached with wt()'s invalidation rules (optimizer step for trained weights, _version
        for writes outside it)."""
        key = (name, count)
        versions, trained = self._group_versions(name, count)
        ent = self._wq.get(key)
        if ent is not None and ent[1] == versions and (not trained or ent[2] == self.opt_epoch):
            return ent[0]
        src = self.fused(name, count, "w") if count > 1 else self.w(name)
        q = ops.mx8_quant(src, *(ent[0] if ent is not None else (None, None)))
        self._wq[key] = (q, versions, self.opt_epoch)
        return q

    def wtq(self, name: str, count: int = 1):
        """Wᵀ as MX-fp8 (e4m3 [in, out] + E8M0 scales [in, out/32], blocks of 32 along `out`): the B
        operand of the opt-in MX-fp8 input-gradient GEMMs dX = dY·W (engine.fp8_bwd).  Quantised
        from wt() and rebuilt whenever wt() rebuilds its transpose."""
        key = (name, count)
        wt = self.wt(name, count)
        ent = self._wtq.get(key)
        if ent is not None and ent[1] is wt and ent[2] == self._wt_stamp.get(key):
            return ent[0]
        q = ops.mx8_quant(wt, *(ent[0] if ent is not None else (None, None)))
        self._wtq[key] = (q, wt, self._wt_stamp.get(key))
        return q

    def w2(self, name: str, count: int = 1):
        """W as [W_bf16 | W_bf16] [out, 2·in] (the B operand of ops.linear_x2: the text encoder's
        precise forward, activations split hi | lo against the bf16 weight twice).  Built from the
        fp32 master; cached with wt()'s invalidation rules; refresh_transposes rebuilds the trained
        ones after an optimizer step."""
        key = (name, count)
        versions, trained = self._group_versions(name, count)
        ent = self._w2.get(key)
        if ent is not None and ent[1] == versions and (not trained or ent[2] == self.opt_epoch):
            self._wait_prebuilt()
            return ent[0]
        s = self.slots[name]
        src = self.master[s.offset:s.offset + s.numel * count].view(s.shape[0] * count, -1)
        dst = ent[0] if ent is not None else None
        if dst is not None:
            self._wait_prebuilt()
        dst = ops.split_bf16(src, 2, 0, dst)
        self._w2[key] = (dst, versions, self.opt_epoch)
        return dst

    def wt2(self, name: str, count: int = 1):
        """[Wᵀ | Wᵀ] bf16 [in, 2·out]: the KC operand of a dX GEMM over a [dy_hi | dy_lo] split image
        (dy to ~fp32 against the bf16 weight).  Rebuilt from wt() whenever that is."""
        wt = self.wt(name, count)
        ent = self._wt2.get((name, count))
        if ent is not None and ent[1] is wt and ent[2] == self._wt_stamp.get((name, count)):
            return ent[0]
        n, k = wt.shape
        dst = ent[0] if ent is not None else torch.empty((n, 2 * k), device=wt.device, dtype=wt.dtype)
        ops.copy2d(dst[:, :k], wt)
        ops.copy2d(dst[:, k:], wt)
        self._wt2[(name, count)] = (dst, wt, self._wt_stamp.get((name, count)))
        return dst

    def wt(self, name: str, count: int = 1):
        """Wᵀ as a contiguous bf16 [in, out] matrix (the KC operand of dX = dY·W; `count` > 1:
        the adjacent fused group starting at `name`, e.g. Q|K|V -> [in, 3·out]).  Built from the
        bf16 shadow by the transpose kernel and cached; rebuilt when the shadow changed: after
        a fused optimizer step for weights that receive gradients, or when a parameter was
        written outside the optimizer (its _version moved)."""
        key = (name, count)
        s = self.slots[name]
        names = [name] if count == 1 else None
        if names is None:
            first = s.offset
            names = [n for n, t in self.slots.items() if first <= t.offset < first + s.numel * count]
        versions = tuple(self.params[n]._version for n in names)
        trained = s.segment in ("enc", "head")
        ent = self._wt.get(key)
        if ent is not None and ent[1] == versions and (not trained or ent[2] == self.opt_epoch):
            self._wait_prebuilt()
            return ent[0]
        src = self.fused(name, count, "w") if count > 1 else self.w(name)
        dst = ent[0] if ent is not None else None
        if dst is not None:
            # the side stream's refresh_transposes may still be writing this buffer: rebuilding
            # it on this stream without the wait would race with that write
            self._wait_prebuilt()
        dst = ops.transpose16(src, dst)
        self._wt[key] = (dst, versions, self.opt_epoch)
        self._wt_stamp[key] = self._wt_stamp.get(key, 0) + 1
        return dst

    def refresh_transposes(self, stream):
        """Rebuild on `stream` every cached Wᵀ of a weight the fused optimizer just updated
        (26 transposes per c2 step), right after the optimizer step, so they overlap the next
        forward instead of sitting on the backward's critical path.  A stream that later takes
        one of them from wt() first waits for this work (one event)."""
        if stream is None or self.device.type != "cuda":
            return
        stale = [k for k, ent in self._wt.items()
                 if ent[2] != self.opt_epoch and self.slots[k[0]].segment in ("enc", "head")]
        stale2 = [k for k, ent in self._w2.items()
                  if ent[2] != self.opt_epoch and self.slots[k[0]].segment in ("enc", "head")]
        if not stale and not stale2:
            return
        cur = torch.cuda.current_stream(self.device)
        stream.wait_stream(cur)               # the optimizer's shadow writes
        self._prebuilt = None                 # the rebuilds below must not wait on the previous event
        with torch.cuda.stream(stream):
            for name, count in stale:
                self.wt(name, count)
            for name, count in stale2:
                self.w2(name, count)
            ev = torch.cuda.Event()
            ev.record(stream)
        self._prebuilt = (ev, stream, set())

    def refresh_transposes_in(self, runs):
        """refresh_transposes for the weights inside the flat-buffer runs [(a, b), ...], on the
        current stream (TrainStep(overlap_optimizer=True): the optimizer stream, right after the
        AdamW of that block, so the block's event covers its transposes too and no consumer waits
        on a global rebuild event)."""
        if self.device.type != "cuda":
            return
        self._prebuilt = None
        inside = lambda k: any(a <= self.slots[k[0]].offset < b for a, b in runs)  # noqa: E731
        for cache, build in ((self._wt, self.wt), (self._w2, self.w2)):
            for k in [k for k, ent in cache.items() if ent[2] != self.opt_epoch
                      and self.slots[k[0]].segment in ("enc", "head") and inside(k)]:
                build(*k)

    def _wait_prebuilt(self):
        pb = getattr(self, "_prebuilt", None)
        if pb is None:
            return
        ev, stream, waited = pb
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream != stream.cuda_stream and cur.cuda_stream not in waited:
            cur.wait_event(ev)
            waited.add(cur.cuda_stream)

    def trainable_layer(self, name: str) -> bool:
        return self.slots[name].segment in ("enc", "head")

    # ----------------------------------------------------------------- shadow
    def sync_shadow(self, force=False):
        """Re-cast the bf16 shadow of any parameter modified outside the fused optimizer."""
        if self.device.type != "cuda":
            return  # meta / cpu stores only serve module-tree inspection; no kernel can run there
        for n, s in self.slots.items():
            v = self.params[n]._version
            if force or self._versions.get(n) != v:
                src = self.master[s.offset:s.offset + s.numel]
                dst = self.shadow[s.offset:s.offset + s.numel]
                ops.cast_bf16(src, dst)
                self._versions[n] = self.params[n]._version

    def mark_synced(self):
        """The fused optimizer refreshed the shadow of every trained parameter."""
        for n in self.slots:
            self._versions[n] = self.params[n]._version
        self.opt_epoch += 1

    # ------------------------------------------------------------------ grads
    def attach_grads(self):
        """Point .grad of every gradient-receiving parameter at its slice of the flat buffer.
        Returns True if the buffer must be zeroed first (grads were reset to None)."""
        reset = False
        for n, s in self.slots.items():
            if s.segment in ("enc", "head"):
                p = self.params[n]
                if p.grad is None:
                    reset = True
        if reset:
            self.grad.zero_()
            for n, s in self.slots.items():
                if s.segment in ("enc", "head"):
                    self.params[n].grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)
        return reset
