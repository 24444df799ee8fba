"""Data-parallel logic on CPU with the gloo backend, world_size 2.

* GradSync (train.py) averages the flat fp32 gradient buffer across ranks: dense blocks as
  bucketed async all-reduces started per backward stage, the word-embedding table by the
  row-sparse (id, row) all-gather.  Its two HIP row kernels are replaced here by torch
  stand-ins (the kernels themselves are checked on the GPU, tests/test_dist_gpu.py).
* The DP design claim — per-rank gradients of equal local batches, averaged, equal the
  global-batch gradient — checked with the oracle's autograd on the golden mini model
  (alignment head on, so the per-sample alignment weighting is covered too).
* EmbeddingExchange (train.py), north_star's all-gather of embeddings before the similarity
  matmul: the global matrix's diagonals are every rank's local s_pos / s_neg, the on-device
  metrics equal the reference's formulas over the global batch, and the optional in-batch
  InfoNCE term (value and both embedding gradients, including the reduce-scattered transcript
  gradient) equals a torch autograd restatement over the global batch.  Its HIP kernels are
  replaced by torch stand-ins here (checked on the GPU in tests/test_dist_gpu.py).
* The layerdrop seed broadcast and the per-rank synthetic data shards.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Store:
    """Minimal ParamStore: grad buffer + named slots (heads / audio / text / word table)."""

    def __init__(self, grad, slots):
        from speech_transcript_embeddings_amd.store import Slot
        self.grad, self.device = grad, grad.device
        self.slots = {n: Slot(n, off, int(np.prod(shape)), shape, seg) for n, off, shape, seg in slots}
        self.n_grad = max(s.offset + s.numel for s in self.slots.values() if s.segment in ("enc", "head"))


def rows_extract_ref(ids, pad, g2, flags, out_ids, rows, count):
    """torch stand-in for ste_rows_extract (test-only)."""
    u = [i for i in dict.fromkeys(ids.tolist()) if i != pad and i >= 0]
    out_ids.fill_(-1)
    rows.zero_()
    out_ids[: len(u)] = torch.tensor(u, dtype=torch.int32)
    rows[: len(u)] = g2[u]
    g2[u] = 0
    count.fill_(len(u))


def rows_accumulate_ref(g2, ids, rows, scale):
    for s, i in enumerate(ids.tolist()):
        if i >= 0:
            g2[i] += rows[s] * scale


class _Recorder:
    """Wraps torch.distributed's collectives while active and records (name, async_op) per call."""
    NAMES = ("all_reduce", "all_gather_into_tensor", "all_gather", "broadcast", "reduce_scatter_tensor", "barrier")

    def __enter__(self):
        self.calls, self._orig = [], {}
        for n in self.NAMES:
            f = self._orig[n] = getattr(dist, n)

            def wrap(*a, _f=f, _n=n, **k):
                self.calls.append((_n, bool(k.get("async_op", False))))
                return _f(*a, **k)
            setattr(dist, n, wrap)
        return self

    def __exit__(self, *exc):
        for n, f in self._orig.items():
            setattr(dist, n, f)


def _sync_case(rank, world):
    """Dense blocks + sparse word table; returns (max err vs the all-rank average, untouched tail ok,
    every collective async).  The ranks hold DIFFERENT token counts (the sparse
    capacity and the sparse-vs-dense choice must still agree): first with the capacity agreed
    for the step by ensure_capacity (MAX over ranks), then with a configured one."""
    from speech_transcript_embeddings_amd import ops
    from speech_transcript_embeddings_amd.train import GradSync
    ops.rows_extract, ops.rows_accumulate = rows_extract_ref, rows_accumulate_ref
    V, D = 50, 4
    slots = [("text_encoder.embeddings.word_embeddings.weight", 0, (V, D), "enc"),
             ("text_encoder.encoder.layer.1.x", 200, (21,), "enc"),
             ("text_encoder.embeddings.LayerNorm.weight", 221, (16,), "enc"),
             ("audio_encoder.encoder.layers.0.x", 240, (101,), "enc"),
             ("audio_encoder.feature_projection.projection.weight", 344, (13,), "enc"),
             ("text_proj.weight", 360, (45,), "head"),
             ("text_encoder.pooler.dense.weight", 408, (9,), "nograd")]

    def local(r):
        g = torch.zeros(417)
        gen = torch.Generator().manual_seed(100 + r)
        for a, b in ((200, 237), (240, 341), (344, 357), (360, 405)):  # dense slots (gaps = alignment padding)
            g[a:b] = torch.randn(b - a, generator=gen)
        ids = torch.randint(2, V, (10 + 2 * r,), generator=gen)
        ids[3] = 1  # padding_idx: never a gradient row
        for i in ids.tolist():
            if i != 1:
                g[i * D:(i + 1) * D] += torch.randn(D, generator=gen)
        return g, ids

    g, ids = local(rank)
    g[408:] = 7.0 + rank  # beyond n_grad: must stay untouched
    expect = sum(local(r)[0] for r in range(world)) / world
    gs = GradSync(_Store(g, slots))
    assert all(gs.ranges[k] for k in GradSync.STAGES), gs.ranges   # every stage has a non-empty block
    gs.bucket = 29  # several buckets + ragged ones
    g0 = g.clone()
    assert gs.ensure_capacity(ids.numel()) == 10 + 2 * (world - 1)   # agreed for the step: the MAX over ranks
    with _Recorder() as rec:
        for stage in GradSync.STAGES:
            gs.stage_done(stage, ids)
    assert gs.sparse is not None and gs.sparse[3] == 10 + 2 * (world - 1)   # sparse, at the agreed capacity
    gs.finish()
    n = gs.store.n_grad
    all_async = bool(rec.calls) and all(a for _, a in rec.calls)
    err = (g[:n] - expect[:n]).abs().max().item()
    # a configured capacity (TrainStep(micro_batch=, max_text_length=)): no agreement collective at all
    g.copy_(g0)
    gs2 = GradSync(_Store(g, slots), word_capacity=12)   # 2 x 12 rows < half the 50-row table: sparse
    gs2.bucket = 29
    with _Recorder() as rec2:
        for stage in GradSync.STAGES:
            gs2.stage_done(stage, ids)
    assert gs2.sparse is not None and gs2.sparse[3] == 12
    gs2.finish()
    err = max(err, (g[:n] - expect[:n]).abs().max().item())
    all_async = all_async and bool(rec2.calls) and all(a for _, a in rec2.calls)
    try:
        gs2.ensure_capacity(13)
        over = False
    except RuntimeError:
        over = True
    assert over, "a step over the configured capacity must raise"
    return err, bool(torch.all(g[408:] == 7.0 + rank)), all_async


def _exchange_stand_ins():
    """torch stand-ins (test-only) for the exchange's HIP kernels."""
    from speech_transcript_embeddings_amd import ops

    def similarity(a, t, S):
        S.copy_(a @ t.t())

    def pair_metrics(S, off_neg, tau, acc, losses=None, loss_w=1.0):
        NB = S.shape[0]
        i = torch.arange(NB)
        sp, sn = S[i, i], S[i, off_neg + i]
        acc[0] += torch.sigmoid(sp / tau).double().sum()
        acc[1] += torch.sigmoid(sn / tau).double().sum()
        acc[2] += (sp > sn).double().sum()
        acc[3] += (S[:, :NB].argmax(1) == i).double().sum()
        acc[4] += NB
        if losses is not None:
            acc[5] += losses.double().sum() * loss_w

    def inbatch_ce(S, B, NB, row0, tau, weight, gscale, loss, dS):
        lg = S[:, :NB] / tau
        tgt = torch.arange(B) + row0
        p = torch.softmax(lg, 1)
        loss += weight / B * torch.nn.functional.cross_entropy(lg, tgt, reduction="sum")
        oh = torch.zeros_like(p)
        oh[torch.arange(B), tgt] = 1.0
        dS.copy_(weight / B * (p - oh) / tau)

    def rowmat(X, Y, out, transpose_x=False):
        out += (X.t() if transpose_x else X) @ Y
        return out

    def axpby(y, x, alpha=1.0, beta=1.0):
        y.mul_(beta).add_(alpha * x)
        return y
    ops.similarity, ops.pair_metrics, ops.inbatch_ce, ops.rowmat, ops.axpby = \
        similarity, pair_metrics, inbatch_ce, rowmat, axpby


def _exchange_case(rank, world):
    import torch.nn.functional as F
    from speech_transcript_embeddings_amd.train import EmbeddingExchange
    _exchange_stand_ins()
    B, P, tau, lam = 3, 8, 0.1, 0.7

    def emb(r):
        g = torch.Generator().manual_seed(500 + r)
        return [F.normalize(torch.randn(B, P, generator=g), dim=1) for _ in range(3)]  # a, tpos, tneg
    a, tp, tn = emb(rank)
    tn_all = torch.cat([tp, tn]).contiguous()
    loss = torch.tensor([0.25 + rank])
    # in_batch_weight == 0 (the reference's loss): start + finish issue only async collectives
    ex0 = EmbeddingExchange(tau)
    with _Recorder() as rec:
        ex0.start(a, tn_all)
        ex0.finish(torch.tensor([0.25 + rank]))
    out_async = bool(rec.calls) and all(x for _, x in rec.calls)
    ex = EmbeddingExchange(tau, in_batch_weight=lam)
    ex.start(a, tn_all)
    # in-batch term (its own loss accumulator and cotangents, zero-initialised)
    lterm = torch.zeros(1)
    dan, dtp = torch.zeros(B, P), torch.zeros(B, P)
    ex.in_batch(a, None, lterm, dan, dtp)
    ex.finish(loss)
    out = {"exchange_async": out_async}
    S = ex.last_S
    NB = world * B
    i = torch.arange(NB)
    local_sp, local_sn = (a * tp).sum(1), (a * tn).sum(1)
    out["diag_ok"] = bool(torch.allclose(S[i, i][rank * B:(rank + 1) * B], local_sp, atol=1e-6) and
                          torch.allclose(S[i, NB + i][rank * B:(rank + 1) * B], local_sn, atol=1e-6))
    # metrics over the global batch, the reference's formulas (ref :1120-1161)
    E = [emb(r) for r in range(world)]
    A_g = torch.cat([e[0] for e in E])
    Tp_g, Tn_g = torch.cat([e[1] for e in E]), torch.cat([e[2] for e in E])
    sp_g, sn_g = (A_g * Tp_g).sum(1), (A_g * Tn_g).sum(1)
    m = ex.epoch_metrics()
    want = {"clean_similarity": torch.sigmoid(sp_g / tau).mean().item(),
            "corrupt_similarity": torch.sigmoid(sn_g / tau).mean().item(),
            "pair_accuracy": (sp_g > sn_g).double().mean().item(),
            "in_batch_top1": ((A_g @ Tp_g.t()).argmax(1) == torch.arange(NB)).double().mean().item(),
            "loss": sum(0.25 + r for r in range(world)) / world}
    out["metrics_ok"] = all(abs(m[k] - v) < 1e-6 for k, v in want.items()) and m["samples"] == NB
    # in-batch term vs autograd over the global batch: rank r's term is lam/B Σ_{i in r} CE_i and
    # its backward cotangents must be d(Σ_r L_r)/d(its own a, tpos) (GradSync then averages)
    Ag = A_g.clone().requires_grad_()
    Tg = Tp_g.clone().requires_grad_()
    lg = Ag @ Tg.t() / tau
    terms = [lam / B * F.cross_entropy(lg[r * B:(r + 1) * B], torch.arange(r * B, (r + 1) * B), reduction="sum")
             for r in range(world)]
    sum(terms).backward()
    out["inbatch_loss_err"] = abs(lterm.item() - terms[rank].item())
    sl = slice(rank * B, (rank + 1) * B)
    out["inbatch_grad_err"] = max((dan - Ag.grad[sl]).abs().max().item(), (dtp - Tg.grad[sl]).abs().max().item())
    return out


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from speech_transcript_embeddings_amd.train import GradSync, TrainStep, synthetic_batch
        from oracle import det_init, ref_model as R
        out = {}
        # 1. overlapped dense all-reduce + row-sparse word table == plain average
        out["sync_err"], out["tail_ok"], out["sync_async"] = _sync_case(rank, world)
        # 2. DP gradient == global-batch gradient (oracle autograd, golden mini model with alignment head)
        meta = json.loads((GOLDEN / "model_golden_align.json").read_text())
        z = np.load(GOLDEN / "model_golden_align.npz")
        keys = ["input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
                "attention_mask_audio"]
        cfg = R.mini_cfg(meta)
        vals = det_init.state_dict_values(R.param_shapes(cfg, spec_augment=False))
        names = list(meta["with_grad"])

        def grads(sl):
            p = {k: torch.from_numpy(v).requires_grad_(k in set(meta["trainable"])) for k, v in vals.items()}
            batch = {k: torch.from_numpy(z[k][sl]) for k in keys}
            loss, *_ = R.step_loss(p, batch, cfg)
            loss.backward()
            return torch.cat([p[k].grad.reshape(-1) for k in names])

        B = z["input_ids_pos"].shape[0]
        per = B // world
        flat = grads(slice(rank * per, (rank + 1) * per)).contiguous()
        dist.all_reduce(flat)
        flat /= world
        full = grads(slice(0, B))
        out["dp_rel"] = ((flat - full).norm() / full.norm()).item()
        # 3. EmbeddingExchange: global similarity matrix, metrics, optional in-batch InfoNCE
        out.update(_exchange_case(rank, world))
        # layerdrop seed: identical draws on every rank
        from speech_transcript_embeddings_amd.train import TrainStep as _TS
        ts = _TS.__new__(_TS)

        class _M:
            class engine:
                layerdrop_gen = None

            class store:
                device = torch.device("cpu")
        ts.model = _M
        ts._sync_layerdrop_seed()
        draws = torch.rand(8, generator=_M.engine.layerdrop_gen)
        alld = [torch.empty_like(draws) for _ in range(world)]
        dist.all_gather(alld, draws)
        out["layerdrop_same"] = all(torch.equal(alld[0], d) for d in alld)
        # 4. per-rank data shards differ (weak scaling: every rank its own local batch)
        wav, lens, ids, *_ = synthetic_batch(2, 4000, 8, device="cpu", rank=rank)
        allw = [torch.empty_like(wav) for _ in range(world)]
        dist.all_gather(allw, wav)
        out["shards_differ"] = not torch.equal(allw[0], allw[1])
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_data_parallel_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=280)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, out in res.items():
        assert out["sync_err"] < 1e-6 and out["tail_ok"], (r, out["sync_err"])
        assert out["sync_async"] and out["exchange_async"], (r, out)   # no synchronous collective in a step
        assert out["dp_rel"] < 1e-5, (r, out["dp_rel"])
        assert out["diag_ok"] and out["metrics_ok"], (r, out)
        assert out["inbatch_loss_err"] < 1e-5 and out["inbatch_grad_err"] < 1e-5, (r, out)
        assert out["layerdrop_same"], r
        assert out["shards_differ"], r



# --------------------------------------------------------------------------------------------
# step_batch holds no host synchronisation at world 2: a TrainStep over a fake
# engine (the forward returns embeddings, the backward finalises the GradSync stages in order)
# with torch stand-ins for the HIP ops.  Every device->host read (item / tolist / cpu / numpy /
# bool / float / int), every stream / event / device synchronize and every blocking collective
# issued from the package's own code is recorded; after the first step there must be none.

class _SyncSpy:
    PKG = "speech_transcript_embeddings_amd"
    READS = ("item", "tolist", "cpu", "numpy", "__bool__", "__float__", "__int__")

    def __enter__(self):
        import sys
        self.hits, self._orig = [], []

        def from_pkg():
            f = sys._getframe(2)
            return self.PKG in f.f_code.co_filename and "test_" not in f.f_code.co_filename

        for name in self.READS:
            orig = getattr(torch.Tensor, name)

            def wrap(t, *a, _o=orig, _n=name, **k):
                if from_pkg():
                    self.hits.append(_n)
                return _o(t, *a, **k)
            self._orig.append((torch.Tensor, name, orig))
            setattr(torch.Tensor, name, wrap)
        for obj, name in ((torch.cuda, "synchronize"), (torch.cuda.Event, "synchronize"),
                          (torch.cuda.Stream, "synchronize"), (torch.cuda.Event, "wait")):
            orig = getattr(obj, name)

            def wrap(*a, _o=orig, _n=name, **k):
                if from_pkg():
                    self.hits.append(_n)
                return _o(*a, **k)
            self._orig.append((obj, name, orig))
            setattr(obj, name, wrap)
        self.rec = _Recorder().__enter__()
        return self

    def __exit__(self, *exc):
        self.rec.__exit__(*exc)
        for obj, name, orig in reversed(self._orig):
            setattr(obj, name, orig)

    def blocking(self):
        return self.hits + [n for n, a in self.rec.calls if not a]


def _fake_model(B, L, P=8, V=50):
    """A model object with the attributes TrainStep / FusedAdamW / GradSync read; the engine's
    forward returns fixed embeddings and its backward writes a gradient per stage."""
    from speech_transcript_embeddings_amd.store import Slot
    slots = [("text_encoder.embeddings.word_embeddings.weight", 0, (V, 4), "enc"),
             ("text_encoder.encoder.layer.1.x", 200, (21,), "enc"),
             ("text_encoder.embeddings.LayerNorm.weight", 221, (16,), "enc"),
             ("audio_encoder.encoder.layers.0.x", 240, (101,), "enc"),
             ("audio_encoder.feature_projection.projection.weight", 344, (13,), "enc"),
             ("text_proj.weight", 360, (45,), "head")]

    class Store:
        device = torch.device("cpu")
        n_grad = 405
        seg_range = {"enc": (0, 357), "head": (357, 405)}

        def __init__(self):
            self.grad = torch.zeros(405)
            self.master = torch.randn(405)
            self.shadow = self.master.clone()
            self.slots = {n: Slot(n, o, int(np.prod(s)), s, g) for n, o, s, g in slots}

        def sync_shadow(self):
            pass

        def mark_synced(self):
            pass

        def refresh_transposes(self, stream=None):
            pass

    class Engine:
        layerdrop_gen = None

        def __init__(self, store):
            self.store = store

        def _side_stream(self):
            return None

        def forward(self, batch, train):
            g = torch.Generator().manual_seed(int(batch["input_ids_pos"].sum()))
            t_ids = torch.cat([batch["input_ids_pos"], batch["input_ids_neg"]])
            e = lambda: torch.randn(B, P, generator=g)  # noqa: E731
            return e(), e(), e(), None, {"t_ids": t_ids}

        def backward(self, ctx, d_tp, d_tn, d_af, d_align, stage_done=None):
            gr = self.store.grad
            gr[360:405] += d_af.sum()
            if stage_done:
                stage_done("heads")
            gr[240:341] += d_tp.sum()
            if stage_done:
                stage_done("audio_layers")
            gr[344:357] += 1.0
            if stage_done:
                stage_done("audio")
            gr[200:221] += d_tn.sum()
            if stage_done:
                stage_done("text_layers")
            gr[221:237] += d_tn.mean()
            for i in ctx["t_ids"].reshape(-1):
                gr[int(i) * 4:int(i) * 4 + 4] += 0.5      # (test code: host reads are fine here)
            if stage_done:
                stage_done("text")

    class Model:
        freeze_encoders = "partial"

        class text_cfg:
            pad_token_id = 1

        def __init__(self):
            self.store = Store()
            self.engine = Engine(self.store)

        def train(self):
            pass
    return Model()


def _head_stand_ins():
    import torch.nn.functional as F
    from speech_transcript_embeddings_amd import ops
    _exchange_stand_ins()

    def l2norm_fwd(x, out, nrm):
        nrm.copy_(x.norm(dim=1))
        out.copy_(F.normalize(x, dim=1))

    def l2norm_bwd(t, nrm, dt, g):
        g.copy_((dt - (dt * t).sum(1, keepdim=True) * t) / nrm[:, None])

    def pair_loss_fwd(S, B, align, B2, L, tau, aw, gamma, sp, sn, loss):
        i = torch.arange(B)
        sp.copy_(S[i, i])
        sn.copy_(S[i, B + i])
        loss.copy_(F.softplus((sn - sp) / tau).mean().view(1))

    def pair_loss_bwd(sp, sn, align, B, L, tau, aw, gamma, gscale, dsp, dsn, dal):
        w = torch.sigmoid((sn - sp) / tau) / (tau * B)
        if gscale is not None:
            w = w * gscale
        dsp.copy_(-w)
        dsn.copy_(w)

    def pair_sim_bwd(an, tp, tn, dsp, dsn, dan, dtp, dtn):
        dan.copy_(dsp[:, None] * tp + dsn[:, None] * tn)
        dtp.copy_(dsp[:, None] * an)
        dtn.copy_(dsn[:, None] * an)

    def sumsq(g, acc, part=None):
        acc += (g.double() ** 2).sum()

    def adamw(master, grad, m, v, shadow, lr, beta1, beta2, eps, wd, step, sumsq_acc=None, max_norm=1.0):
        clip = torch.clamp(max_norm / (sumsq_acc.sqrt() + 1e-6), max=1.0).float() if sumsq_acc is not None else 1.0
        g = grad * clip
        m.mul_(beta1).add_((1 - beta1) * g)
        v.mul_(beta2).add_((1 - beta2) * g * g)
        master.sub_(lr * (m / (v.sqrt() + eps) + wd * master))
        shadow.copy_(master)
    ops.l2norm_fwd, ops.l2norm_bwd, ops.pair_loss_fwd, ops.pair_loss_bwd, ops.pair_sim_bwd = \
        l2norm_fwd, l2norm_bwd, pair_loss_fwd, pair_loss_bwd, pair_sim_bwd
    ops.sumsq, ops.adamw = sumsq, adamw
    ops.rows_extract, ops.rows_accumulate = rows_extract_ref, rows_accumulate_ref


def _nosync_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from speech_transcript_embeddings_amd.train import TrainStep
        _head_stand_ins()
        B, L = 3, 4
        out = {}
        for mode in ("configured", "agreed_per_step"):
            for acc in (1, 2):
                model = _fake_model(B, L)
                kw = dict(micro_batch=B, max_text_length=L) if mode == "configured" else {}
                step = TrainStep(model, warmup=1, total_steps=10, accumulation_steps=acc, in_batch_weight=0.3, **kw)
                g = torch.Generator().manual_seed(10 + rank)
                hits = []
                for it in range(3 * acc):
                    ids = torch.randint(2, 50, (B, L), generator=g)
                    neg = torch.randint(2, 50, (B, L), generator=g)
                    batch = {"input_ids_pos": ids, "attention_mask_pos": torch.ones(B, L, dtype=torch.long),
                             "input_ids_neg": neg, "attention_mask_neg": torch.ones(B, L, dtype=torch.long)}
                    with _SyncSpy() as spy:
                        step.step_batch(batch)
                    # the unconfigured capacity is agreed on every optimizer step's final
                    # micro-batch, before any of its work is queued (a capacity agreed
                    # once goes stale when a later step carries more ids); nothing else blocks
                    agree = mode == "agreed_per_step" and it % acc == acc - 1
                    if not agree:
                        hits += spy.blocking()
                out[f"{mode}/acc{acc}"] = hits
                out[f"{mode}/acc{acc}/steps"] = step.opt.t
                out[f"{mode}/acc{acc}/finite"] = bool(torch.isfinite(model.store.master).all())
        q.put((rank, out))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_step_batch_no_host_sync_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_nosync_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=170)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, out in res.items():
        assert "error" not in out, out.get("error")
        for mode in ("configured", "agreed_per_step"):
            for acc in (1, 2):
                k = f"{mode}/acc{acc}"
                assert out[k] == [], (r, k, out[k])      # no host read, no sync, no blocking collective
                assert out[k + "/steps"] == 3 and out[k + "/finite"], (r, k)
