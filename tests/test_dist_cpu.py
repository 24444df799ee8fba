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
    capacity and the sparse-vs-dense choice must still agree), agreed by plan_words."""
    from speech_transcript_embeddings_amd import ops
    from speech_transcript_embeddings_amd.train import GradSync
    ops.rows_extract, ops.rows_accumulate = rows_extract_ref, rows_accumulate_ref
    V, D = 50, 4
    slots = [("text_encoder.embeddings.word_embeddings.weight", 0, (V, D), "enc"),
             ("text_encoder.encoder.layer.1.x", 200, (37,), "enc"),
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
    with _Recorder() as rec:
        gs.plan_words(ids.numel())
        for stage in GradSync.STAGES:
            gs.stage_done(stage, ids)
    assert gs.sparse is not None and gs.sparse[3] == 10 + 2 * (world - 1)   # sparse, at the agreed MAX capacity
    gs.finish()
    n = gs.store.n_grad
    all_async = bool(rec.calls) and all(a for _, a in rec.calls)
    return (g[:n] - expect[:n]).abs().max().item(), bool(torch.all(g[408:] == 7.0 + rank)), all_async


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

