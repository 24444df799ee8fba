"""Data-parallel path on the GPU: the row-sparse exchange kernels against torch, and two
gloo ranks sharing cuda:0 running full TrainStep steps through GradSync (overlapped dense
all-reduces + sparse word-embedding exchange): the replicas must stay bit-identical and the
averaged gradient must equal the mean of the two local gradients."""
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
        from test_model_gpu import load, mini_model
        from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
        meta, _ = load("align")
        model = mini_model(meta)
        step = TrainStep(model, warmup=1, total_steps=10)
        data = synthetic_batch(2, 16000, 12, vocab=1000, rank=rank)
        st = model.store
        loss = step(*data).item()
        torch.cuda.synchronize()
        out = {"loss": loss}
        master = st.master.clone()
        allm = [torch.empty_like(master) for _ in range(world)]
        dist.all_gather(allm, master)
        out["replicas_equal"] = all(torch.equal(allm[0], m) for m in allm)
        out["finite"] = bool(torch.isfinite(master).all())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


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
        r, out = q.get(timeout=220)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, out in res.items():
        assert out["replicas_equal"] and out["finite"], (r, out)
    assert res[0]["loss"] != res[1]["loss"]  # different local shards
