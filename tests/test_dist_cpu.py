"""Data-parallel logic on CPU with the gloo backend, world_size 2.

* GradSync (train.py) averages the flat fp32 gradient buffer across ranks: dense blocks as
  bucketed async all-reduces started per backward stage, the word-embedding table by the
  row-sparse (id, row) all-gather.  Its two HIP row kernels are replaced here by torch
  stand-ins (the kernels themselves are checked on the GPU, tests/test_dist_gpu.py).
* The DP design claim — per-rank gradients of equal local batches, averaged, equal the
  global-batch gradient — checked with the oracle's autograd on the golden mini model
  (alignment head on, so the per-sample alignment weighting is covered too).
* The embedding all-gather used for global similarity metrics and the per-rank synthetic
  data shards.
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


def _sync_case(rank, world):
    """Dense blocks + sparse word table; returns (max err vs the all-rank average, untouched tail ok)."""
    from speech_transcript_embeddings_amd import ops
    from speech_transcript_embeddings_amd.train import GradSync
    ops.rows_extract, ops.rows_accumulate = rows_extract_ref, rows_accumulate_ref
    V, D = 50, 4
    slots = [("text_encoder.embeddings.word_embeddings.weight", 0, (V, D), "enc"),
             ("text_encoder.encoder.layer.1.x", 200, (37,), "enc"),
             ("audio_encoder.encoder.layers.0.x", 240, (101,), "enc"),
             ("text_proj.weight", 344, (61,), "head"),
             ("text_encoder.pooler.dense.weight", 408, (9,), "nograd")]

    def local(r):
        g = torch.zeros(417)
        gen = torch.Generator().manual_seed(100 + r)
        for a, b in ((200, 237), (240, 341), (344, 405)):  # the dense slots (gaps = alignment padding)
            g[a:b] = torch.randn(b - a, generator=gen)
        ids = torch.randint(2, V, (12,), generator=gen)
        ids[3] = 1  # padding_idx: never a gradient row
        for i in ids.tolist():
            if i != 1:
                g[i * D:(i + 1) * D] += torch.randn(D, generator=gen)
        return g, ids

    g, ids = local(rank)
    g[408:] = 7.0 + rank  # beyond n_grad: must stay untouched
    expect = sum(local(r)[0] for r in range(world)) / world
    gs = GradSync(_Store(g, slots))
    gs.bucket = 29  # several buckets + ragged ones
    for stage in GradSync.STAGES:
        gs.stage_done(stage, ids)
    gs.finish()
    n = gs.store.n_grad
    return (g[:n] - expect[:n]).abs().max().item(), bool(torch.all(g[408:] == 7.0 + rank))


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
        out["sync_err"], out["tail_ok"] = _sync_case(rank, world)
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
        # 3. embedding all-gather for global metrics
        ts = TrainStep.__new__(TrainStep)
        ts.last = {}
        an = torch.full((3, 4), float(rank))
        tn = torch.full((6, 4), float(10 + rank))
        ts._gather_metrics(an, tn)
        ga, gt = ts.last["global_emb"]
        out["gather_ok"] = all(torch.equal(ga[r], torch.full((3, 4), float(r))) for r in range(world)) and \
            all(torch.equal(gt[r], torch.full((6, 4), float(10 + r))) for r in range(world))
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
        assert out["dp_rel"] < 1e-5, (r, out["dp_rel"])
        assert out["gather_ok"], r
        assert out["shards_differ"], r

