"""The fused training step and its optimizer tail, single GPU or data-parallel.

One step (the body of ref:training/trainer_unfreeze.py:train_epoch, ref:1057-1117, with
accumulation_steps micro-batches per optimizer step, 1 by default):
    GPU fbank from raw waveforms (replaces the 12 CPU DataLoader workers' extractor calls)
 -> forward (engine.py)  -> L2-normalise -> B x 2B similarity on the fp32 MFMA
 -> AlignmentAwareInfoNCE -> backward (engine.py)
 -> [DP] RCCL all-reduce (average) of the dense gradient blocks, each started as soon as the
    backward has finished it, plus a row-sparse exchange of the word-embedding gradient
 -> clip_grad_norm_(1.0) + two-group AdamW + linear warmup schedule, fused in HBM.

Data parallel: the loss is a mean of per-sample terms, so averaging
per-rank gradients of equal local batches equals the global-batch gradient exactly;
the only collectives are the gradient all-reduce and a small all-gather of the
normalised embeddings (global similarity metrics; optional in-batch negatives).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from . import _lib, ops
from .model import EnhancedAudioTextModel

F32 = torch.float32


class LinearWarmupSchedule:
    """transformers.get_linear_schedule_with_warmup (ref:1537-1541); lr(0) = 0."""

    def __init__(self, warmup: int, total: int):
        self.warmup, self.total, self.step_count = warmup, total, 0

    def factor(self, step=None):
        s = self.step_count if step is None else step
        if s < self.warmup:
            return s / max(1, self.warmup)
        return max(0.0, (self.total - s) / max(1, self.total - self.warmup))

    def step(self):
        self.step_count += 1


class FusedAdamW:
    """torch.optim.AdamW over the reference's param groups with clip_grad_norm_(max_norm)
    (ref:1108) folded in: one Σg² pass, then one AdamW pass per group that reads the clip
    coefficient on device (no host sync).  Groups (ref:1486-1519): freeze_encoders="partial"
    -> encoder params at lr/50 and the rest at lr; any other mode -> one group at lr.
    weight_decay 0.01, betas (0.9, 0.999), eps 1e-8.

    state_dict() / load_state_dict() use torch.optim.AdamW's format with the reference's
    parameter numbering, so optimizer states move between this optimizer and a reference
    AdamW in either direction (checkpoint parity)."""

    def __init__(self, model: EnhancedAudioTextModel, lr=2.1e-3, encoder_lr_div=50.0, weight_decay=0.01,
                 betas=(0.9, 0.999), eps=1e-8, max_norm=1.0):
        st = model.store
        self.model = model
        self.store = st
        self.partial = getattr(model, "freeze_encoders", "partial") == "partial"
        div = encoder_lr_div if self.partial else 1.0
        self.groups = [{"range": st.seg_range["enc"], "lr": lr / div},
                       {"range": st.seg_range["head"], "lr": lr}]
        self.wd, self.betas, self.eps, self.max_norm = weight_decay, betas, eps, max_norm
        self.exp_avg = torch.zeros(st.n_grad, device=st.device, dtype=F32)
        self.exp_avg_sq = torch.zeros(st.n_grad, device=st.device, dtype=F32)
        self.sumsq = torch.zeros(1, device=st.device, dtype=torch.float64)
        self.sumsq_part = torch.zeros(ops.SUMSQ_PARTS, device=st.device, dtype=torch.float64)  # ordered Σg²
        self.t = 0
        self.last_factor = 1.0
        # the event after the last update when it ran on another stream (TrainStep's
        # overlap_optimizer): every host-side read or write of the optimizer's buffers waits on it
        self.tail = None

    def sync(self):
        """Order the current stream after the last update (a no-op when it ran on this stream)."""
        if self.tail is not None:
            torch.cuda.current_stream(self.store.device).wait_event(self.tail)

    # ------------------------------------------------------- torch.optim format
    def _ref_groups(self):
        """The reference's param groups as lists of parameter names (ref:1494-1519)."""
        named = [(n, p) for n, p in self.model.named_parameters() if p.requires_grad]
        if not self.partial:
            return [[n for n, _ in named]]
        enc = [n for n, _ in named if "text_encoder" in n or "audio_encoder" in n]
        rest = [n for n, _ in named if not ("text_encoder" in n or "audio_encoder" in n)]
        return [enc, rest]

    def _group_hparams(self, gi):
        base = self.groups[0]["lr"] if (self.partial and gi == 0) else self.groups[1]["lr"]
        return {"lr": base * self.last_factor, "weight_decay": self.wd, "betas": tuple(self.betas), "eps": self.eps,
                "amsgrad": False, "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
                "fused": None, "decoupled_weight_decay": True, "initial_lr": base}

    def state_dict(self, lr_factor: float | None = None):
        """torch.optim.AdamW.state_dict() layout: per-parameter {"step", "exp_avg", "exp_avg_sq"}
        for every parameter that has received a gradient step (none before the first step),
        keyed by the reference's parameter index; param_groups carry lr = initial_lr x
        lr_factor (default: the factor of the last step; LambdaLR leaves the NEXT step's factor
        there, which TrainStep.optimizer_state_dict() passes) and initial_lr."""
        if lr_factor is not None:
            saved, self.last_factor = self.last_factor, lr_factor
            try:
                return self.state_dict()
            finally:
                self.last_factor = saved
        self.sync()
        st = self.store
        state, groups, idx = {}, [], 0
        for gi, names in enumerate(self._ref_groups()):
            ids = []
            for n in names:
                s = st.slots[n]
                if self.t > 0 and s.segment in ("enc", "head"):
                    sl = slice(s.offset, s.offset + s.numel)
                    state[idx] = {"step": torch.tensor(float(self.t), dtype=F32),
                                  "exp_avg": self.exp_avg[sl].view(s.shape).clone(),
                                  "exp_avg_sq": self.exp_avg_sq[sl].view(s.shape).clone()}
                ids.append(idx)
                idx += 1
            groups.append({**self._group_hparams(gi), "params": ids})
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """Inverse of state_dict(); accepts a reference AdamW state_dict of the same model
        configuration (same parameter numbering).  Restores the moments, the step count, the
        base learning rates (initial_lr, or lr without a scheduler) and the shared
        betas / eps / weight decay."""
        st = self.store
        self.sync()   # the moments are rewritten below: after the last update has read them
        ref = self._ref_groups()
        pgs = sd["param_groups"]
        if len(pgs) != len(ref) or any(len(g["params"]) != len(r) for g, r in zip(pgs, ref)):
            raise ValueError("optimizer state_dict does not match this model's parameter groups "
                             f"({[len(g['params']) for g in pgs]} vs {[len(r) for r in ref]})")
        steps = set()
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        for g, names in zip(pgs, ref):
            for i, n in zip(g["params"], names):
                ps = sd["state"].get(i)
                if ps is None:
                    continue
                s = st.slots[n]
                if s.segment not in ("enc", "head"):
                    continue  # a parameter the HIP backward never produces a gradient for
                sl = slice(s.offset, s.offset + s.numel)
                self.exp_avg[sl].copy_(ps["exp_avg"].reshape(-1).to(self.exp_avg.device, F32))
                self.exp_avg_sq[sl].copy_(ps["exp_avg_sq"].reshape(-1).to(self.exp_avg_sq.device, F32))
                steps.add(int(float(ps["step"])))
        if len(steps) > 1:
            raise ValueError(f"parameters at different step counts {sorted(steps)}: not supported by the fused "
                             "optimizer (one shared step)")
        self.t = steps.pop() if steps else 0
        bases = [g.get("initial_lr", g["lr"]) for g in pgs]
        if self.partial:
            self.groups[0]["lr"], self.groups[1]["lr"] = bases[0], bases[1]
            self.last_factor = pgs[1]["lr"] / bases[1] if bases[1] else 1.0
        else:
            self.groups[0]["lr"] = self.groups[1]["lr"] = bases[0]
            self.last_factor = pgs[0]["lr"] / bases[0] if bases[0] else 1.0
        g0 = pgs[0]
        self.wd, self.betas, self.eps = float(g0["weight_decay"]), tuple(g0["betas"]), float(g0["eps"])

    def total_norm(self):
        """clip_grad_norm_'s return value for the last step (the pre-clip global gradient norm);
        reads the on-device Σg² (host sync), after the update that produced it (overlap_optimizer:
        another stream, which the current one would not otherwise wait for)."""
        self.sync()
        return math.sqrt(float(self.sumsq.item()))

    def step(self, lr_factor: float = 1.0, phases=None, on_phase=None):
        """Clip + AdamW.  phases: [(name, [(a, b), ...]), ...] — the update split into flat-buffer
        runs launched phase by phase, with a CUDA event recorded after each (returned as
        {name: event}), so the next forward can wait for just the parameters it is about to read
        (TrainStep(overlap_optimizer=True)).  AdamW is elementwise, so the split changes no value;
        each run takes its group's learning rate from the segment it lies in; on_phase(runs) runs
        after each phase's update, before its event (the block's cached transposes)."""
        st = self.store
        self.t += 1
        self.last_factor = lr_factor
        self.sumsq.zero_()
        if self.max_norm is not None:
            ops.sumsq(st.grad[: st.n_grad], self.sumsq, self.sumsq_part)

        def upd(a, b, lr):
            ops.adamw(st.master[a:b], st.grad[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b], st.shadow[a:b],
                      lr=lr * lr_factor, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, wd=self.wd,
                      step=self.t, sumsq_acc=self.sumsq if self.max_norm is not None else None,
                      max_norm=self.max_norm or 1.0)
        events = {}
        if phases is None:
            for gr in self.groups:
                a, b = gr["range"]
                if b > a:
                    upd(a, b, gr["lr"])
            st.mark_synced()
            return events
        st.mark_synced()   # first: on_phase sees this step's weights as the ones to rebuild from
        for name, runs in phases:
            for a, b in runs:
                gr = next(g for g in self.groups if g["range"][0] <= a and b <= g["range"][1])
                upd(a, b, gr["lr"])
            if on_phase is not None:
                on_phase(runs)
            ev = torch.cuda.Event()
            ev.record()
            events[name] = ev
        return events

    def zero_grad(self):
        self.sync()   # the last update has read the gradients
        self.store.grad.zero_()


class GradSync:
    """Data-parallel gradient averaging, overlapped with the backward.

    The flat gradient buffer is split into the blocks the backward finishes in order
    (STAGES), and engine.backward calls stage_done(name) as each becomes final:
      "heads"         after the heads' backward (before either encoder's);
      "audio_layers"  the trainable Conformer layers, once the backward has passed the lowest of
                      them (the frozen layers' input-gradient passes still run behind it);
      "audio"         the rest of the audio encoder (feature projection, SpecAugment embedding),
                      at the end of the audio backward;
      "text_layers"   the trainable XLM-R layers, once the text backward has passed the lowest
                      of them (the frozen text layers' input-gradient passes still run behind it);
      "text"          the rest of the text encoder (embedding LayerNorm, position and token-type
                      tables, the word table), at the end of the text backward.
    The text stages are signalled from the side stream the text backward runs on (that stream
    current), so their collectives queue behind the text backward alone and overlap the audio
    backward (on one stream: after the audio backward).
    Each block's dense ranges are all-reduced asynchronously (RCCL ring over xGMI, <= bucket_mb
    per call, average) while the remaining backward kernels run.  The 250,002 x 768
    word-embedding gradient is exchanged row-sparse: each rank extracts the rows of its own token
    ids (ste_rows_extract), all-gathers fixed-capacity (id, row) lists and adds every rank's list in
    rank order (ste_rows_accumulate), so every rank ends with the same averaged dense gradient an
    all-reduce would give, from ~2*b*L rows instead of 192 M values.  When the lists would not be
    smaller than the table (world x capacity >= vocab / 2, e.g. long accumulation windows), the
    table goes through the dense all-reduce instead.
    The list capacity, and with it the sparse-vs-dense choice, must be identical on every rank
    (one rank in all_gather while another is in all_reduce hangs the job), but ranks may hold
    different token counts (a short last batch, length-bucketed padding).  The capacity is fixed
    per run, never agreed per step: word_capacity = the most token ids one optimizer step can
    carry (TrainStep: 2 x micro-batch x max_text_length x accumulation; the reference pads every
    transcript to max_text_length, ref :838-851); a step with more ids than a configured capacity
    raises on every rank alike only if every rank's count exceeds it, so the configured value must
    be a true bound.  When the caller cannot say, the capacity is agreed on EVERY optimizer step by
    start_capacity() (a MAX all-reduce that TrainStep starts before the step's kernels are queued,
    on a stream of its own, read back at the text stage), so ranks with different token counts
    (length-bucketed padding) always take the same path.  A step's backward therefore holds no
    collective of its own and no host wait on the step's streams.
    `finish()` waits for every collective (on the current stream) before clip + AdamW.
    """

    WORDS = "text_encoder.embeddings.word_embeddings.weight"
    # in the order the backward finalises them: the heads; the trainable Conformer layers (the
    # top k, final once the backward has passed the lowest of them, while the frozen layers'
    # input gradients still run); the rest of the audio encoder (feature projection, SpecAugment
    # embedding: final at the very end); the trainable text layers (side stream, final once its
    # backward has passed the lowest of them); the rest of the text encoder (end of the text backward)
    STAGES = ("heads", "audio_layers", "audio", "text_layers", "text")

    def __init__(self, store, bucket_mb: int = 256, pad_id: int = 1, word_capacity: int | None = None):
        self.store = store
        self.bucket = max(1, bucket_mb * 1024 * 1024 // 4)
        self.pad_id = pad_id
        self.works = []
        self.sparse = None
        self.capacity = None if word_capacity is None else int(word_capacity)
        self.configured = word_capacity is not None
        self._agreed = False   # unconfigured: the capacity was agreed for the current step
        self._pending_cap = None   # start_capacity()'s (event, pinned host value, device value)
        self._cap_stream = None
        grad_slots = [sl for sl in store.slots.values() if sl.segment in ("enc", "head")]

        ordered = sorted(grad_slots, key=lambda x: x.offset)

        def span(pred):
            """The contiguous runs of matching slots in buffer order (a slot of another block
            ends a run), so a block never swallows another block's slots."""
            runs, cur = [], None
            for x in ordered:
                if pred(x):
                    cur = [x.offset, x.offset + x.numel] if cur is None else [cur[0], x.offset + x.numel]
                elif cur is not None:
                    runs.append(tuple(cur))
                    cur = None
            if cur is not None:
                runs.append(tuple(cur))
            return runs

        words = store.slots.get(self.WORDS)
        self.words = words if words is not None and words.segment == "enc" else None
        self.ranges = {"heads": span(lambda x: x.segment == "head"),
                       "audio_layers": span(lambda x: x.segment == "enc" and
                                            x.name.startswith("audio_encoder.encoder.layers.")),
                       "audio": span(lambda x: x.segment == "enc" and x.name.startswith("audio_encoder.") and
                                     not x.name.startswith("audio_encoder.encoder.layers.")),
                       "text_layers": span(lambda x: x.segment == "enc" and
                                           x.name.startswith("text_encoder.encoder.layer.")),
                       "text": span(lambda x: x.segment == "enc" and x.name.startswith("text_encoder.") and
                                    not x.name.startswith("text_encoder.encoder.layer."))}
        if self.words is not None and self.ranges["text"]:
            w0, w1 = self.words.offset, self.words.offset + self.words.numel
            cut = []
            for a, b in self.ranges["text"]:
                cut += [r for r in ((a, min(b, w0)), (max(a, w1), b)) if r[1] > r[0]] if a < w1 and w0 < b else [(a, b)]
            self.ranges["text"] = cut
        # the blocks must not overlap, and every gradient slot must lie inside exactly one block
        # (a slot no block covers would never be synchronised and the replicas would drift)
        cov = sorted(r for rs in self.ranges.values() for r in rs)
        for (a0, b0), (a1, b1) in zip(cov, cov[1:]):
            assert b0 <= a1, "gradient blocks overlap"
        for x in grad_slots:
            if self.words is not None and x.name == self.WORDS:
                continue
            inside = [k for k, rs in self.ranges.items()
                      if any(a <= x.offset and x.offset + x.numel <= b for a, b in rs)]
            assert len(inside) == 1, f"gradient slot {x.name} is in {len(inside)} sync blocks"
        self._flags = None

    @staticmethod
    def active():
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def _avg_op(self):
        return dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM

    def _reduce(self, ranges):
        g = self.store.grad
        ws = dist.get_world_size()
        op = self._avg_op()
        for a, b in ranges:
            for c in range(a, b, self.bucket):
                t = g[c:min(b, c + self.bucket)]
                if op == dist.ReduceOp.SUM:
                    t.mul_(1.0 / ws)
                self.works.append(dist.all_reduce(t, op=op, async_op=True))

    def ensure_capacity(self, n_ids: int) -> int:
        """The step's word-table exchange capacity.  Configured: checked (raises when a step
        carries more ids).  Not configured: the MAX of every rank's n_ids, agreed with a blocking
        all-reduce (TrainStep uses start_capacity(), which does not block the host)."""
        if not self.active() or self.words is None:
            return int(n_ids)
        if not self.configured:
            dev = self.store.device
            t = torch.tensor([int(n_ids)], dtype=torch.int64,
                             device=dev if dist.get_backend() == "nccl" and dev.type == "cuda" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            self.capacity = int(t.item())
            self._agreed = True
            self._pending_cap = None
        elif n_ids > self.capacity:
            raise RuntimeError(f"{n_ids} token ids in one step exceed the word-table exchange capacity "
                               f"{self.capacity} (TrainStep(micro_batch=, max_text_length=) sets it)")
        return self.capacity

    def start_capacity(self, n_ids: int):
        """ensure_capacity() without a host wait, for TrainStep: made once per optimizer step before
        the step's kernels are queued.  Not configured, on RCCL: the MAX all-reduce runs on a stream
        of its own (nothing queued there to wait for) and its result is copied to pinned host memory
        under an event, which the text stage reads (resolve) — so the host keeps running ahead of
        the GPU instead of draining the previous step at every step start.  Gloo (host
        tensors) and configured capacities: ensure_capacity() itself."""
        if not self.active() or self.words is None:
            return
        dev = self.store.device
        if self.configured or not (dist.get_backend() == "nccl" and dev.type == "cuda"):
            self.ensure_capacity(n_ids)
            return
        if self._cap_stream is None:
            self._cap_stream = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(self._cap_stream):
            t = torch.tensor([int(n_ids)], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, async_op=True).wait()   # this stream waits for it
            host = torch.empty(1, dtype=torch.int64, pin_memory=True)
            host.copy_(t, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self._pending_cap = (ev, host, t)
        self._agreed = True

    def _agreed_capacity(self) -> int:
        if self._pending_cap is not None:
            ev, host, _ = self._pending_cap
            ev.synchronize()
            self.capacity = int(host.item())
            self._pending_cap = None
        return self.capacity

    def _sparse_words(self, ids, cap_ids):
        st, sl = self.store, self.words
        D = sl.shape[1]
        g2 = st.grad[sl.offset:sl.offset + sl.numel].view(sl.shape)
        dev = st.device
        if self._flags is None:
            self._flags = torch.zeros(sl.shape[0], device=dev, dtype=torch.int32)
        cap = min(cap_ids, sl.shape[0])
        out_ids = torch.empty(cap, device=dev, dtype=torch.int32)
        rows = torch.empty(cap, D, device=dev, dtype=F32)
        count = torch.empty(1, device=dev, dtype=torch.int32)
        ops.rows_extract(ids, self.pad_id, g2, self._flags, out_ids, rows, count)
        ws = dist.get_world_size()
        all_ids = torch.empty(ws * cap, device=dev, dtype=torch.int32)
        all_rows = torch.empty(ws * cap, D, device=dev, dtype=F32)
        w1 = dist.all_gather_into_tensor(all_ids, out_ids, async_op=True)
        w2 = dist.all_gather_into_tensor(all_rows, rows, async_op=True)
        self.sparse = (g2, all_ids, all_rows, cap, ws, (w1, w2), (out_ids, rows))

    def sparse_pays(self, n_ids: int) -> bool:
        """Row-sparse word-table exchange only while world x capacity rows stay well below the
        table (with long accumulation windows the (id, row) lists outgrow a dense
        all-reduce of the 250,002 x 768 table)."""
        ws = dist.get_world_size()
        return ws * min(n_ids, self.words.shape[0]) < self.words.shape[0] // 2

    def stage_done(self, stage, ids=None):
        if not self.active():
            return
        self._reduce(self.ranges[stage])
        if stage == "text" and self.words is not None:
            if self.configured or not self._agreed:
                n = self.ensure_capacity(ids.numel() if ids is not None else 0)
            else:   # agreed for this step before its kernels were queued
                n = self._agreed_capacity()
            self._agreed = False
            if ids is not None and self.sparse_pays(n):   # n, hence the choice, equal on every rank
                self._sparse_words(ids, n)
            else:
                self._reduce([(self.words.offset, self.words.offset + self.words.numel)])

    def finish(self):
        for w in self.works:
            w.wait()
        self.works = []
        if self.sparse is not None:
            g2, all_ids, all_rows, cap, ws, waits, keep = self.sparse
            for w in waits:
                w.wait()
            if all_ids.is_cuda:   # made on the stream that ran the text backward, read here
                cur = torch.cuda.current_stream(all_ids.device)
                for t in (all_ids, all_rows, *keep):
                    t.record_stream(cur)
            for r in range(ws):  # rank order: identical summation on every rank
                ops.rows_accumulate(g2, all_ids[r * cap:(r + 1) * cap], all_rows[r * cap:(r + 1) * cap], 1.0 / ws)
            self.sparse = None


class EmbeddingExchange:
    """north_star's "RCCL all-gather of embeddings over xGMI before the similarity matmul"
    (SURVEY §8e, D1).

    start() (after the forward): the L2-normalised audio, clean and corrupted transcript
    embeddings [B, P] of every rank are all-gathered asynchronously into A_g [NB, P] and
    T_g = [Tpos_g; Tneg_g] [2NB, P] (NB = ranks x B); the collective runs on RCCL's stream
    while the local loss and the backward proceed.
    finish() (after the backward): waits, forms the global similarity matrix
    S_g = A_g·T_gᵀ [NB, 2NB] on the fp32 MFMA (its diagonals are every rank's s_pos / s_neg,
    the reference's per-sample logits, ref :1073-1074) and accumulates the reference's epoch
    metrics on the device (ref train_epoch :1120-1161: sample-weighted loss, clean / corrupt
    similarity as sigmoid(s/0.1), gap) plus the pair accuracy and the in-batch top-1 retrieval
    rate; epoch_metrics() syncs them to the host once.
    Optional in-batch negatives (in_batch_weight > 0; 0 by default = the reference's loss): the
    gather is awaited before the loss, the local rows S = A·Tpos_gᵀ [B, NB] feed an InfoNCE over
    all NB clean transcripts of the global batch (target: the sample's own), the audio gradient
    is dS·Tpos_g and the transcript gradient dSᵀ·A is reduce-scattered (sum) to the owning
    ranks before their L2-normalise backward.  With one process the same code runs without
    collectives (NB = B)."""

    # tests: run the collective branches even on a one-rank group (the RCCL path on one GPU)
    FORCE_COLLECTIVES = False

    def __init__(self, tau: float = 0.1, in_batch_weight: float = 0.0):
        self.tau, self.weight = float(tau), float(in_batch_weight)
        self.acc = None
        self.steps = 0
        self._pending = None

    @staticmethod
    def world():
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(), dist.get_rank()
        return 1, 0

    def _collective(self, ws):
        return ws > 1 or (self.FORCE_COLLECTIVES and dist.is_available() and dist.is_initialized())

    def start(self, an, tn_all):
        ws, rank = self.world()
        B, P = an.shape
        NB = ws * B
        if not self._collective(ws):
            self._pending = (an, tn_all, [], B, 1, 0)
            return
        A_g = torch.empty(NB, P, device=an.device, dtype=F32)
        T_g = torch.empty(2 * NB, P, device=an.device, dtype=F32)
        works = [dist.all_gather_into_tensor(A_g, an, async_op=True),
                 dist.all_gather_into_tensor(T_g[:NB], tn_all[:B], async_op=True),
                 dist.all_gather_into_tensor(T_g[NB:], tn_all[B:], async_op=True)]
        self._pending = (A_g, T_g, works, B, ws, rank)

    def _wait(self):
        A_g, T_g, works, B, ws, rank = self._pending
        for w in works:
            w.wait()
        self._pending = (A_g, T_g, [], B, ws, rank)
        return A_g, T_g, B, ws, rank

    def in_batch(self, an, gscale, loss, dan, dtp):
        """Adds the in-batch InfoNCE value to loss and its gradients to dan / dtp (the cotangents of
        the local normalised audio / clean transcript embeddings)."""
        A_g, T_g, B, ws, rank = self._wait()
        NB = ws * B
        e = lambda *sh: torch.empty(sh, device=an.device, dtype=F32)  # noqa: E731
        S = e(B, NB)
        ops.similarity(an, T_g[:NB], S)
        dS = e(B, NB)
        ops.inbatch_ce(S, B, NB, rank * B, self.tau, self.weight, gscale, loss, dS)
        ops.rowmat(dS, T_g[:NB], dan)                      # d a_i   += Σ_j dS_ij t_j
        dT = torch.zeros(NB, an.shape[1], device=an.device, dtype=F32)
        ops.rowmat(dS, an, dT, transpose_x=True)           # d t_j   += Σ_i dS_ij a_i (every rank's t_j)
        if self._collective(ws):
            if dist.get_backend() == "gloo" and dT.is_cuda:   # gloo reduce-scatters host tensors only
                mine = torch.empty(B, an.shape[1], dtype=F32)
                dist.reduce_scatter_tensor(mine, dT.cpu(), op=dist.ReduceOp.SUM, async_op=True).wait()
                mine = mine.to(dT.device)
            else:
                # RCCL: wait() only makes the current stream wait for the collective's stream
                mine = e(B, an.shape[1])
                dist.reduce_scatter_tensor(mine, dT, op=dist.ReduceOp.SUM, async_op=True).wait()
            ops.axpby(dtp, mine)
        else:
            ops.axpby(dtp, dT)

    def finish(self, loss):
        """Global similarity matrix + on-device metric accumulation (after the backward).  No
        collective here: the similarity metrics come from the gathered embeddings (identical on
        every rank), and acc[5] sums only this rank's B·loss; epoch_metrics() all-reduces it once
        per epoch."""
        if self._pending is None:
            return
        A_g, T_g, B, ws, rank = self._wait()
        self._pending = None
        NB = ws * B
        dev = A_g.device
        if self.acc is None:
            self.acc = torch.zeros(6, device=dev, dtype=torch.float64)
        S = torch.empty(NB, 2 * NB, device=dev, dtype=F32)
        ops.similarity(A_g, T_g, S)
        ops.pair_metrics(S, NB, self.tau, self.acc, losses=loss, loss_w=float(B))
        self.last_S = S
        self.steps += 1

    def epoch_metrics(self, reset: bool = True):
        """The reference's train_epoch return keys (ref :1156-1162) over the global batch, plus
        pair_accuracy (s_pos > s_neg) and in_batch_top1 (retrieval among the clean transcripts).
        One device->host transfer; with several ranks also one all-reduce of the loss sum, so
        every rank must call it (at the same epoch boundary)."""
        ws, _ = self.world()
        if self.acc is None:
            if ws > 1:   # keep the collective matched with ranks that did accumulate
                raise RuntimeError("epoch_metrics() before any finish() on this rank")
            return {}
        a = self.acc.cpu().tolist()
        if ws > 1:
            # the global loss sum is used for the returned value only: acc[5] keeps this rank's own
            # sum, so a later call (reset=False, or accumulation continuing) never re-reduces a total
            lsum = self.acc[5:6].clone()
            if dist.get_backend() == "gloo" and lsum.is_cuda:
                lsum = lsum.cpu()
            dist.all_reduce(lsum, op=dist.ReduceOp.SUM)
            a[5] = float(lsum.item())
        n = a[4]
        if n == 0:
            return {}
        out = {"loss": a[5] / n, "clean_similarity": a[0] / n, "corrupt_similarity": a[1] / n,
               "similarity_gap": (a[0] - a[1]) / n, "pair_accuracy": a[2] / n, "in_batch_top1": a[3] / n,
               "samples": int(n)}
        if reset:
            self.acc.zero_()
        return out


class TrainStep:
    """fbank -> forward -> loss -> backward -> all-reduce -> clip + AdamW (+ schedule)."""

    def __init__(self, model: EnhancedAudioTextModel, lr=2.1e-3, warmup=100, total_steps=10000, temperature=0.1,
                 alignment_weight=0.5, corrupt_gamma=0.35, max_norm=1.0, pad_value=1.0, gather_embeddings=True,
                 accumulation_steps=1, in_batch_weight=0.0, micro_batch=None, max_text_length=None,
                 overlap_optimizer=False):
        """accumulation_steps (ref train_epoch :1064-1117): each call is one micro-batch whose loss
        gradient is scaled by 1/accumulation_steps and summed into the flat gradient buffer; the
        data-parallel sync, clip, AdamW and scheduler step run on every accumulation_steps-th
        call (the sync overlapped with that micro-batch's backward) and on flush(), the
        reference's `is_last_batch` step after a partial window.
        gather_embeddings: the EmbeddingExchange (global similarity matrix + on-device epoch
        metrics); in_batch_weight > 0 adds its optional in-batch-negative InfoNCE term (0 keeps
        the reference's loss exactly).
        Data parallel: rank 0's layerdrop seed is broadcast so every rank drops the same Conformer
        layers (tf:…wav2vec2_bert…:519-522 draws one number per layer per batch).  micro_batch and
        max_text_length (the reference pads transcripts to it, ref :838-851) fix the word-table
        exchange capacity (GradSync) up front; without them it is agreed on every optimizer step.
        overlap_optimizer (CUDA): clip + AdamW run on a stream of their own, split into the
        parameter blocks the next forward reads in order — the feature projection first, then the
        text encoder, then the trainable Conformer layers and the heads — and that forward waits
        for each block right before its first read, so the update of the late blocks overlaps the
        fbank and the frozen Conformer layers.  Parameters read outside the step between steps
        (checkpointing, evaluation on another stream): call sync() first."""
        self.model = model
        self.acc = max(1, int(accumulation_steps))
        self._micro = 0
        self._ids = []
        self.opt = FusedAdamW(model, lr=lr, max_norm=max_norm)
        self.sched = LinearWarmupSchedule(warmup, total_steps)
        cap = None
        if micro_batch is not None and max_text_length is not None:
            cap = 2 * int(micro_batch) * int(max_text_length) * self.acc   # clean + corrupted ids per window
        self.gradsync = GradSync(model.store, pad_id=model.text_cfg.pad_token_id, word_capacity=cap)
        self.tau, self.aw, self.gamma = temperature, alignment_weight, corrupt_gamma
        self.pad_value = pad_value
        self.gather_embeddings = gather_embeddings or in_batch_weight > 0
        self.exchange = EmbeddingExchange(temperature, in_batch_weight) if self.gather_embeddings else None
        self.in_batch_weight = float(in_batch_weight)
        self.last = {}
        st = model.store
        self.overlap = bool(overlap_optimizer) and st.device.type == "cuda"
        self._opt_stream = torch.cuda.Stream(device=st.device) if self.overlap else None
        self._opt_tail = None
        if self.overlap:
            gs = self.gradsync
            text = gs.ranges["text"] + gs.ranges["text_layers"]
            if gs.words is not None:
                text = text + [(gs.words.offset, gs.words.offset + gs.words.numel)]
            self._phases = [("audio", gs.ranges["audio"]), ("text", sorted(text)),
                            ("late", gs.ranges["audio_layers"] + gs.ranges["heads"])]
        self._sync_layerdrop_seed()

    def _sync_layerdrop_seed(self):
        seed = torch.randint(0, 2**62, (1,), dtype=torch.int64)
        if GradSync.active():
            t = seed.to(self.model.store.device) if dist.get_backend() == "nccl" else seed.clone()
            dist.broadcast(t, src=0)
            seed = t.cpu()
        self.model.engine.layerdrop_gen = torch.Generator().manual_seed(int(seed.item()))

    def features(self, wav, lengths):
        """GPU fbank for a batch of raw 16 kHz waveforms -> (input_values, attention_mask_audio).
        wav2vec2 audio encoder: Wav2Vec2FeatureExtractor's per-clip normalisation instead
        (ste_w2v_wave_norm) and the sample mask of the clip lengths."""
        if self.model.engine.raw_audio:
            from .wav2vec2 import wave_normalize
            B, n = wav.shape
            lengths = lengths.to(device=wav.device, dtype=torch.int32)
            mask = (torch.arange(n, device=wav.device).view(1, n) < lengths.view(B, 1)).to(torch.int64)
            return wave_normalize(wav, lengths), mask
        n = int(wav.shape[1])
        T = ((1 + (n - 400) // 160) + 1) // 2
        lengths = lengths.to(device=wav.device, dtype=torch.int32, non_blocking=True)
        return ops.fbank(wav, lengths, T, pad_value=self.pad_value, mask_mode=0)

    def __call__(self, wav, lengths, ids_pos, mask_pos, ids_neg, mask_neg):
        """One micro-batch from raw 16 kHz waveforms (GPU fbank first).  lengths on the host (as a
        DataLoader delivers them) also give SpecAugment its per-clip frame counts with no
        device->host sync; on the device they are read back only if SpecAugment is on."""
        host = lengths.tolist() if lengths.device.type == "cpu" else None
        feats, amask = self.features(wav, lengths)
        batch = {"input_ids_pos": ids_pos, "attention_mask_pos": mask_pos, "input_ids_neg": ids_neg,
                 "attention_mask_neg": mask_neg, "input_values": feats, "attention_mask_audio": amask}
        if host is not None:
            from .features import num_frames
            batch["audio_lengths"] = host if self.model.engine.raw_audio else [num_frames(int(x)) for x in host]
        return self.step_batch(batch)

    def step_batch(self, batch):
        """One micro-batch given the reference's collated batch dict (custom_collate_fn layout,
        ref :913-921: input_values are features), on the GPU."""
        m = self.model
        m.train()
        st = m.store
        st.sync_shadow()
        eng = m.engine
        if self._micro + 1 == self.acc:   # the window's last micro-batch: check the word-table exchange
            # capacity (agreed across ranks here if not configured) before any kernel is queued
            n_ids = batch["input_ids_pos"].numel() + batch["input_ids_neg"].numel()
            self.gradsync.start_capacity(n_ids + sum(int(t.numel()) for t in (self._ids if self._micro else [])))
        tf_p, tf_n, af, align, ctx = eng.forward(batch, True)
        B, P = af.shape
        # L2 normalise, similarity matrix S = A·[Tp;Tn]^T (fp32 MFMA), loss on its diagonals
        e = lambda *s: torch.empty(s, device=st.device, dtype=F32)  # noqa: E731
        tn_all = e(2 * B, P)
        an = e(B, P)
        nrm = e(3 * B)
        ops.l2norm_fwd(tf_p, tn_all[:B], nrm[:B])
        ops.l2norm_fwd(tf_n, tn_all[B:], nrm[B:2 * B])
        ops.l2norm_fwd(af, an, nrm[2 * B:])
        S = e(B, 2 * B)
        ops.similarity(an, tn_all, S)
        sp, sn, loss = e(B), e(B), e(1)
        L = align.shape[1] if align is not None else 0
        ops.pair_loss_fwd(S, B, align, B, L, self.tau, self.aw, self.gamma, sp, sn, loss)
        if self.exchange is not None:
            self.exchange.start(an, tn_all)   # async all-gather of the embeddings (overlaps the backward)
        # backward
        dsp, dsn = e(B), e(B)
        dal = e(B, L) if align is not None else None
        gscale = None if self.acc == 1 else torch.full((1,), 1.0 / self.acc, device=st.device, dtype=F32)
        ops.pair_loss_bwd(sp, sn, align, B, L, self.tau, self.aw, self.gamma, gscale, dsp, dsn, dal)
        dan, dtp, dtn = e(B, P), e(B, P), e(B, P)
        ops.pair_sim_bwd(an, tn_all[:B], tn_all[B:], dsp, dsn, dan, dtp, dtn)
        if self.in_batch_weight > 0:
            self.exchange.in_batch(an, gscale, loss, dan, dtp)
        g_tp, g_tn, g_a = e(B, P), e(B, P), e(B, P)
        ops.l2norm_bwd(tn_all[:B], nrm[:B], dtp, g_tp)
        ops.l2norm_bwd(tn_all[B:], nrm[B:2 * B], dtn, g_tn)
        ops.l2norm_bwd(an, nrm[2 * B:], dan, g_a)
        if self._micro == 0:
            self._await_optimizer()   # the previous step's AdamW has read these gradients
            st.grad.zero_()
            self._ids = []
        self._ids.append(ctx["t_ids"].reshape(-1))
        self._micro += 1
        final = self._micro == self.acc
        ids_all = self._ids[0] if len(self._ids) == 1 else torch.cat(self._ids)
        eng.backward(ctx, g_tp, g_tn, g_a, dal,
                     stage_done=(lambda stg: self.gradsync.stage_done(stg, ids_all)) if final else None)
        self.last = {"loss": loss, "s_pos": sp, "s_neg": sn}
        if self.exchange is not None:
            self.exchange.finish(loss)
        if final:
            self._optimizer_step()
        return loss

    def epoch_metrics(self):
        """train_epoch's return dict (ref :1156-1162) over the global batch, synced once."""
        self._await_optimizer()
        out = self.exchange.epoch_metrics() if self.exchange is not None else {}
        out["optimizer_steps"] = self.opt.t
        return out

    def _optimizer_step(self):
        eng = self.model.engine
        if self.overlap:
            main = torch.cuda.current_stream(self.model.store.device)
            self._opt_stream.wait_stream(main)
            with torch.cuda.stream(self._opt_stream):
                self.gradsync.finish()
                # each block's cached transposes rebuilt right after its update, under its event
                eng.param_events = self.opt.step(self.sched.factor(), phases=self._phases,
                                                 on_phase=self.model.store.refresh_transposes_in)
                self.sched.step()
                self._opt_tail = torch.cuda.Event()
                self._opt_tail.record()
            self.opt.tail = self._opt_tail
        else:
            self.gradsync.finish()
            self.opt.step(self.sched.factor())  # reference order: optimizer.step() then scheduler.step()
            self.sched.step()
            # the updated weights' cached Wᵀ (dX GEMM operands) rebuild on the side stream, under
            # the next forward
            self.model.store.refresh_transposes(eng._side_stream())
        self._micro = 0
        self._ids = []

    def _await_optimizer(self):
        if self._opt_tail is not None:
            torch.cuda.current_stream(self.model.store.device).wait_event(self._opt_tail)

    def sync(self):
        """Order the current stream after the last optimizer step (overlap_optimizer): parameters,
        moments and gradients are then safe to read or write on it."""
        self._await_optimizer()

    def flush(self):
        """Step on a partial accumulation window (ref :1064-1066 `is_last_batch`): sync the
        accumulated gradients (not overlapped: the backward already ran), clip, AdamW, schedule.
        Returns whether a step was taken."""
        if self._micro == 0:
            return False
        ids_all = torch.cat(self._ids)
        for stg in GradSync.STAGES:
            self.gradsync.stage_done(stg, ids_all)
        self._optimizer_step()
        return True

    def optimizer_state_dict(self):
        """The optimizer state as the reference's training loop would save it after this many
        optimizer.step(); scheduler.step() pairs (group lr = the next step's scheduled lr)."""
        self._await_optimizer()
        return self.opt.state_dict(lr_factor=self.sched.factor())

    def load_optimizer_state_dict(self, sd):
        """Restore moments + step count and put the warmup schedule at the same step."""
        self._await_optimizer()
        self.opt.load_state_dict(sd)
        self.sched.step_count = self.opt.t


def synthetic_batch(B, n_samples, L, vocab=250000, device="cuda", seed=0, rank=0):
    """SURVEY §8d synthetic inputs: 0.1·N(0,1) + 3 sinusoids waveforms, ids ~ U[5, vocab) with
    BOS=0 / EOS=2, full masks, corrupted = 20% of positions re-drawn.  Built on the GPU."""
    g = torch.Generator(device=device).manual_seed(seed * 1000 + rank)
    t = torch.arange(n_samples, device=device, dtype=F32) / 16000.0
    wav = 0.1 * torch.randn(B, n_samples, device=device, generator=g)
    freqs = 100 + 2900 * torch.rand(B, 3, 1, device=device, generator=g)
    wav = wav + 0.05 * torch.sin(2 * math.pi * freqs * t.view(1, 1, -1)).sum(1)
    wav = wav.clamp_(-1, 1).contiguous()
    lengths = torch.full((B,), n_samples, device=device, dtype=torch.int32)
    ids = torch.randint(5, vocab, (B, L), device=device, generator=g)
    ids[:, 0], ids[:, -1] = 0, 2
    corrupt = torch.rand(B, L, device=device, generator=g) < 0.2
    corrupt[:, 0] = False
    corrupt[:, -1] = False
    neg = torch.where(corrupt, torch.randint(5, vocab, (B, L), device=device, generator=g), ids)
    mask = torch.ones(B, L, device=device, dtype=torch.int64)
    return wav, lengths, ids, mask, neg.contiguous(), mask.clone()


__all__ = ["TrainStep", "FusedAdamW", "LinearWarmupSchedule", "GradSync", "EmbeddingExchange", "synthetic_batch",
           "_lib"]
