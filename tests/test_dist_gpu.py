"""Data-parallel path on the GPU: the row-sparse exchange kernels against torch, and two
gloo ranks sharing cuda:0 running full TrainStep steps through GradSync (dense all-reduces
launched mid-backward per stage, the trainable Conformer layers' one while the frozen layers'
input gradients still run, + the sparse word-embedding exchange) and the EmbeddingExchange
(SURVEY §8e):
  * the GradSync-averaged gradient buffer equals the mean of the two ranks' local gradients
    (each computed by the same step with the sync disabled), block by block;
  * after an optimizer step the replicas are bit-identical;
  * the global similarity matrix's diagonals are the ranks' s_pos / s_neg, and the optional
    in-batch InfoNCE term (real kernels, reduce-scattered transcript gradient) matches a torch
    restatement over the global batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_rows_extract_accumulate():
    from speech_transcript_embeddings_amd import ops
    torch.manual_seed(0)
    V, D, n = 1000, 64, 300
    g = torch.randn(V, D, device="cuda")
    ids = torch.randint(0, 200, (n,), device="cuda")
    ids[::7] = 1  # padding_idx
    flags = torch.zeros(V, device="cuda", dtype=torch.int32)
    out_ids = torch.empty(n, device="cuda", dtype=torch.int32)
    rows = torch.empty(n, D, device="cuda")
    count = torch.empty(1, device="cuda", dtype=torch.int32)
    g0 = g.clone()
    ops.rows_extract(ids, 1, g, flags, out_ids, rows, count)
    u = sorted(set(ids.tolist()) - {1})
    got = out_ids[out_ids >= 0].tolist()
    assert sorted(got) == u and len(got) == len(set(got)) == int(count.item())
    assert torch.all(out_ids[len(u):] == -1) and torch.all(flags == 0)
    sel = out_ids[: len(u)].long()
    assert torch.equal(rows[: len(u)], g0[sel]) and torch.all(rows[len(u):] == 0)
    assert torch.all(g[sel] == 0)
    keep = torch.ones(V, dtype=torch.bool, device="cuda")
    keep[sel] = False
    assert torch.equal(g[keep], g0[keep])
    ops.rows_accumulate(g, out_ids, rows, 0.5)
    ref = g0.clone()
    ref[sel] *= 0.5
    assert torch.equal(g, ref)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _body(rank, world, q)
    except Exception:  # report instead of leaving the parent waiting on the queue
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


def _body(rank, world, q):
    import torch.nn.functional as F
    from test_model_gpu import load, mini_model
    from speech_transcript_embeddings_amd import train as TR
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    meta, _ = load("align")

    def build():
        m = mini_model(meta, spec_augment=False)
        m.dropout = 0.0   # a deterministic function, so the synced and local runs compare
        m.audio_cfg.conformer_conv_dropout = 0.0
        m.text_cfg.hidden_dropout_prob = 0.0
        m.text_cfg.attention_probs_dropout_prob = 0.0
        return m
    data = synthetic_batch(2, 16000, 12, vocab=1000, rank=rank)
    out = {}
    # local gradient: the same step with the data-parallel sync switched off (lr 0: no update)
    m_loc = build()
    active = TR.GradSync.__dict__["active"]   # the staticmethod object itself
    TR.GradSync.active = staticmethod(lambda: False)
    try:
        TrainStep(m_loc, lr=0.0, warmup=1, total_steps=10)(*data)
    finally:
        TR.GradSync.active = active
    torch.cuda.synchronize()
    g_loc = m_loc.store.grad[: m_loc.store.n_grad].clone()
    # synced step
    model = build()
    step = TrainStep(model, lr=0.0, warmup=1, total_steps=10)
    loss = step(*data).item()
    torch.cuda.synchronize()
    st = model.store
    g_avg = st.grad[: st.n_grad].clone()
    allg = [torch.empty_like(g_loc) for _ in range(world)]
    dist.all_gather(allg, g_loc)
    mean = sum(allg) / world
    errs = {}
    for stage, rs in step.gradsync.ranges.items():
        for a, b in rs:
            d = (g_avg[a:b] - mean[a:b]).norm() / (mean[a:b].norm() + 1e-30)
            errs[stage] = max(errs.get(stage, 0.0), d.item())
    w = st.slots[TR.GradSync.WORDS]
    sl = slice(w.offset, w.offset + w.numel)
    errs["word_embeddings"] = ((g_avg[sl] - mean[sl]).norm() / mean[sl].norm()).item()
    errs["all"] = ((g_avg - mean).norm() / mean.norm()).item()
    out["avg_errs"] = errs
    out["loss"] = loss
    # an optimizer step: replicas stay identical
    step2 = TrainStep(model, lr=1e-3, warmup=1, total_steps=10)
    step2(*data)
    torch.cuda.synchronize()
    master = st.master.clone()
    allm = [torch.empty_like(master) for _ in range(world)]
    dist.all_gather(allm, master)
    out["replicas_equal"] = all(torch.equal(allm[0], m_) for m_ in allm)
    out["finite"] = bool(torch.isfinite(master).all())
    # global similarity matrix vs the local diagonals
    S = step2.exchange.last_S
    B = data[0].shape[0]
    NB = world * B
    i = torch.arange(NB, device=S.device)
    sp, sn = step2.last["s_pos"], step2.last["s_neg"]
    out["diag_err"] = max((S[i, i][rank * B:(rank + 1) * B] - sp).abs().max().item(),
                          (S[i, NB + i][rank * B:(rank + 1) * B] - sn).abs().max().item())
    out["metrics"] = step2.epoch_metrics()
    # in-batch InfoNCE on the real kernels vs a torch restatement over the global batch
    from speech_transcript_embeddings_amd.train import EmbeddingExchange
    g = torch.Generator(device="cuda").manual_seed(900 + rank)
    a, tp, tn = (F.normalize(torch.randn(B, 64, device="cuda", generator=g), dim=1) for _ in range(3))
    ex = EmbeddingExchange(0.1, in_batch_weight=0.5)
    ex.start(a, torch.cat([tp, tn]).contiguous())
    lterm = torch.zeros(1, device="cuda")
    dan, dtp = torch.zeros(B, 64, device="cuda"), torch.zeros(B, 64, device="cuda")
    ex.in_batch(a, None, lterm, dan, dtp)
    torch.cuda.synchronize()
    A_g = [torch.empty_like(a) for _ in range(world)]
    T_g = [torch.empty_like(tp) for _ in range(world)]
    dist.all_gather(A_g, a)
    dist.all_gather(T_g, tp)
    Ag = torch.cat(A_g).double().requires_grad_()
    Tg = torch.cat(T_g).double().requires_grad_()
    lg = Ag @ Tg.t() / 0.1
    terms = [0.5 / B * F.cross_entropy(lg[r * B:(r + 1) * B], torch.arange(r * B, (r + 1) * B, device="cuda"),
                                       reduction="sum") for r in range(world)]
    sum(terms).backward()
    sl = slice(rank * B, (rank + 1) * B)
    out["inbatch_err"] = max(abs(lterm.item() - terms[rank].item()),
                             (dan.double() - Ag.grad[sl]).abs().max().item(),
                             (dtp.double() - Tg.grad[sl]).abs().max().item())
    q.put((rank, out))


@pytest.mark.timeout(240)
def test_trainstep_two_ranks_gloo_same_gpu():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=150)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, out in res.items():
        print(r, out)
        assert "error" not in out, out.get("error")
        assert out["replicas_equal"] and out["finite"], (r, out)
        # fp32 summation order of atomically accumulated gradients: identical to ~1e-6
        assert all(e < 1e-5 for e in out["avg_errs"].values()), (r, out["avg_errs"])
        assert set(out["avg_errs"]) >= {"heads", "audio_layers", "audio", "text_layers", "text", "word_embeddings"}
        assert out["diag_err"] < 1e-5, (r, out["diag_err"])
        assert out["inbatch_err"] < 1e-4, (r, out["inbatch_err"])
        assert out["metrics"]["samples"] == 4 and out["metrics"]["optimizer_steps"] == 1
    assert res[0]["metrics"] == res[1]["metrics"]  # computed from the same global matrix
    assert res[0]["loss"] != res[1]["loss"]  # different local shards
