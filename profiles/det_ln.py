"""LayerNorm backward-pair determinism under a concurrent stream (GPU diagnosis tooling).

Runs ste_layernorm_bwd_pair REPS times on identical inputs (c2 rows: 3,992 x 1024), with the
second stream idle, busy with our GEMM + attention, or busy with a torch matmul; reports the
repetitions whose outputs differ from the first one, where, and whether the inputs changed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speech_transcript_embeddings_amd import ops  # noqa: E402

BF16, F32 = torch.bfloat16, torch.float32
dev = "cuda"
M, D = 3992, 1024
REPS = int(os.environ.get("REPS", "40"))
g = torch.Generator(device=dev).manual_seed(0)


def rn(*s, dt=BF16, sc=1.0):
    return (torch.randn(*s, device=dev, generator=g) * sc).to(dt)


busy = torch.cuda.Stream()
bx, bw = rn(2048, 768), rn(3072, 768, sc=0.02)
bqkv = rn(2048, 2304)
bo = torch.empty(2048, 768, device=dev, dtype=BF16)
blse = torch.empty(32 * 12 * 64, device=dev)
ta = rn(4096, 4096)


def load(mode, n=40):
    if mode == "idle":
        return
    busy.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(busy):
        for _ in range(n):
            if mode in ("ours", "gemm"):
                ops.linear(bx, bw, out_bf16=True)
            if mode in ("ours", "attn"):
                ops.attention_fwd(bqkv[:, :768], bqkv[:, 768:1536], bqkv[:, 1536:], B=32, T=64, H=12, o=bo,
                                  lse=blse)
            if mode == "torch":
                torch.mm(ta, ta)


x = rn(M, D, dt=F32)
gam = 1 + 0.1 * rn(D, dt=F32)
bet = 0.1 * rn(D, dt=F32)
st = ops.layernorm_fwd(x, gam, bet, 1e-5, yb=torch.empty(M, D, device=dev, dtype=BF16))
dy = rn(M, D)
dres = rn(M, D, dt=F32)
inputs = [x, gam, bet, st[0], st[1], dy, dres]
in0 = [t.clone() for t in inputs]
MODES = os.environ.get("MODES", "idle,gemm,attn,torch").split(",")
NAMES = ["dx", "dxb", "dx0", "dg", "db", "ds", "dg2", "db2"]


def pair(reduce=True):
    dx = torch.empty(M, D, device=dev)
    dxb = torch.empty(M, D, device=dev, dtype=BF16)
    dx0 = torch.empty(M, D, device=dev)
    sums = [torch.zeros(D, device=dev) for _ in range(5)]
    dg, db, ds, dg2, db2 = sums if reduce else (None,) * 5
    first = dict(x=x, mean=st[0], rstd=st[1], gamma=gam, beta=bet, dgamma=dg2, dbeta=db2, dres=dres, dx=dx0)
    second = dict(dy=dy, x=x, mean=st[0], rstd=st[1], gamma=gam, beta=bet, dx=dx, dxb=dxb, dgamma=dg, dbeta=db,
                  dsum=ds, out_scale=0.5)
    ops.layernorm_bwd_pair(first, second)
    return [dx, dxb, dx0] + (sums if reduce else [])


def single():
    dx = torch.empty(M, D, device=dev)
    dxb = torch.empty(M, D, device=dev, dtype=BF16)
    dg, db, ds = (torch.zeros(D, device=dev) for _ in range(3))
    ops.layernorm_bwd(dy, x, st[0], st[1], gam, beta=bet, dx=dx, dxb=dxb, dres=dres, dgamma=dg, dbeta=db, dsum=ds)
    return [dx, dxb, dg, db, ds]


for name, fn in (("pair", pair), ("pair_noreduce", lambda: pair(False)), ("single", single)):
    for mode in MODES:
        ref = None
        nbad = 0
        for r in range(REPS):
            load(mode)
            out = fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = [t.clone() for t in out]
                continue
            diff = [(NAMES[i] if name.startswith("pair") else i, int((t != ref[i]).sum())) for i, t in enumerate(out)
                    if not torch.equal(t, ref[i])]
            if diff:
                nbad += 1
                if nbad <= 3:
                    k = 0 if not torch.equal(out[0], ref[0]) else 2   # b's dx, else a's dx0
                    bad = (out[k] != ref[k]).nonzero()[:20].tolist()
                    vals = [(float(ref[k][i, j]), float(out[k][i, j])) for i, j in bad[:6]]
                    print(f"  {name}/{mode} rep {r}: {diff} out[{k}] at {bad} ref/got {vals}", flush=True)
        changed = [i for i, (a, b) in enumerate(zip(inputs, in0)) if not torch.equal(a, b)]
        print(f"{name}/{mode}: {nbad}/{REPS - 1} repetitions differ; inputs changed: {changed}", flush=True)
