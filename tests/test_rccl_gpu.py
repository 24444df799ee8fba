"""The RCCL branches of the data-parallel step, executed on the one-GPU box.

A freshly spawned child creates a world-size-1 RCCL communicator before any GPU call
(`init_process_group("nccl", device_id=...)`, the form bench.py uses at N > 1), forces
GradSync and EmbeddingExchange onto their collective branches (a one-rank group normally skips
them) and runs one full-dims TrainStep (w2v-bert-2.0 Conformer + XLM-R, B = 2, 10 s clips,
64 tokens) with the optional in-batch InfoNCE term on.  Checked:
  * the device-buffer collectives ran on RCCL: ReduceOp.AVG all-reduces of the dense gradient
    blocks, all_gather_into_tensor (embedding exchange, sparse word-table rows) and
    reduce_scatter_tensor (the in-batch term's transcript gradient), all on CUDA tensors;
  * the synced gradient buffer equals the local one bit for bit: every dense block and the
    word-table slice are snapshotted (on the step's stream) right before their collective is
    enqueued, and compared after GradSync.finish() — a one-rank AVG / gather / reduce-scatter /
    row re-accumulation must be the identity;
  * the word-table capacity is the configured one (no per-step agreement collective); without
    one, the per-step MAX agreement is a single asynchronous all-reduce (GradSync.start_capacity).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(port, q):
    import sys
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        # before any other GPU call: the communicator binds cuda:0 eagerly
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from speech_transcript_embeddings_amd import train as TR
        from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
        out = {"backend": dist.get_backend()}
        calls = []
        orig = {n: getattr(dist, n) for n in ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor",
                                              "broadcast")}

        def wrap(name):
            def f(*a, **k):
                t = a[0] if a else k.get("tensor")
                op = k.get("op")
                calls.append((name, str(op) if op is not None else None, bool(getattr(t, "is_cuda", False)),
                              bool(k.get("async_op", False))))
                return orig[name](*a, **k)
            return f
        for n in orig:
            setattr(dist, n, wrap(n))
        TR.GradSync.active = staticmethod(lambda: True)
        TR.EmbeddingExchange.FORCE_COLLECTIVES = True

        torch.manual_seed(0)
        model = EnhancedAudioTextModel(device="cuda", spec_augment=False)
        B, N, L = 2, 160000, 64
        step = TR.TrainStep(model, lr=1e-3, warmup=1, total_steps=10, in_batch_weight=0.3, micro_batch=B,
                            max_text_length=L)
        gs = step.gradsync
        snaps = []
        reduce0, sparse0 = gs._reduce, gs._sparse_words

        def reduce_snap(ranges):
            for a, b in ranges:
                snaps.append(((a, b), gs.store.grad[a:b].clone()))
            return reduce0(ranges)

        def sparse_snap(ids, cap):
            w = gs.words
            snaps.append(((w.offset, w.offset + w.numel), gs.store.grad[w.offset:w.offset + w.numel].clone()))
            out["sparse_cap"] = cap
            return sparse0(ids, cap)
        gs._reduce, gs._sparse_words = reduce_snap, sparse_snap
        data = TR.synthetic_batch(B, N, L, device="cuda", seed=1)
        loss = step(*data)
        torch.cuda.synchronize()
        out["loss_finite"] = bool(torch.isfinite(loss).all())
        g = gs.store.grad
        covered = sum(b - a for (a, b), _ in snaps)
        out["covered"] = covered
        out["n_grad"] = gs.store.n_grad
        out["bitwise"] = all(torch.equal(g[a:b], s) for (a, b), s in snaps)
        out["nonzero"] = bool(g[: gs.store.n_grad].abs().sum() > 0)
        out["calls"] = list(calls)
        out["metrics"] = step.epoch_metrics()
        # capacity NOT configured: agreed per optimizer step by an async MAX all-reduce on a stream of
        # its own (GradSync.start_capacity), read back at the text stage without a host drain
        del calls[:]
        step2 = TR.TrainStep(model, lr=1e-3, warmup=1, total_steps=10)
        gs2, caps = step2.gradsync, []
        sparse2 = gs2._sparse_words
        gs2._sparse_words = lambda ids, cap: (caps.append(cap), sparse2(ids, cap))[1]
        out["loss2_finite"] = bool(torch.isfinite(step2(*data)).all())
        torch.cuda.synchronize()
        out["calls2"], out["caps2"] = list(calls), caps
        q.put(out)
    except Exception:
        import traceback
        q.put({"error": traceback.format_exc()})
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_rccl_world1_full_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=540)
    p.join(timeout=60)
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    calls = out["calls"]
    print("collectives:", sorted({(n, op, cuda, a) for n, op, cuda, a in calls}))
    assert all(cuda for _, _, cuda, _ in calls), calls
    avg = [c for c in calls if c[0] == "all_reduce" and c[1] is not None and "AVG" in c[1]]
    assert len(avg) >= 4, calls                          # dense blocks: heads, audio layers, audio, text
    assert any(c[0] == "all_gather_into_tensor" for c in calls)
    assert any(c[0] == "reduce_scatter_tensor" for c in calls)
    assert not any(c[0] == "all_reduce" and c[1] is not None and "MAX" in c[1] for c in calls)  # no capacity plan
    assert out["sparse_cap"] == 2 * 2 * 64
    assert out["bitwise"], "one-rank RCCL collectives changed the gradient"
    # every gradient slot went through a snapshotted collective (word table included)
    assert out["covered"] >= 0.95 * out["n_grad"], (out["covered"], out["n_grad"])
    assert out["nonzero"] and out["loss_finite"]
    assert out["metrics"]["samples"] == 2 and out["metrics"]["optimizer_steps"] == 1
    # unconfigured capacity: one asynchronous MAX all-reduce per optimizer step, the agreed value used
    assert [c for c in out["calls2"] if c[0] == "all_reduce" and c[1] is not None and "MAX" in c[1]] == \
        [("all_reduce", str(torch.distributed.ReduceOp.MAX), True, True)], out["calls2"]
    assert out["caps2"] == [2 * 2 * 64] and out["loss2_finite"]
