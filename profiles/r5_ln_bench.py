"""Isolated LayerNorm forward / backward at c2 rows (31,936 x 1,024): HIP-event time per launch
and checksums (A/B variants of a load-policy change must agree bit for bit)."""
import json
import sys
import torch
sys.path.insert(0, ".")
from speech_transcript_embeddings_amd import ops

M, D = 31936, 1024
torch.manual_seed(0)
x = torch.randn(M, D, device="cuda")
gm = torch.rand(D, device="cuda") + 0.5
bt = torch.randn(D, device="cuda") * 0.1
yb = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
mean = torch.empty(M, device="cuda")
rstd = torch.empty(M, device="cuda")
dy = torch.randn(M, D, device="cuda").bfloat16()
dres = torch.randn(M, D, device="cuda")
dx = torch.empty(M, D, device="cuda")


def fwd():
    ops.layernorm_fwd(x, gm, bt, 1e-5, yb=yb, mean=mean, rstd=rstd)


def bwd():
    ops.layernorm_bwd(dy, x, mean, rstd, gm, dx=dx, dres=dres)


res = {}
for name, f in (("fwd", fwd), ("bwd", bwd)):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) * 1e3 / 50, 2)
res["checksum"] = [float(yb.float().sum()), float(dx.double().sum())]
print(json.dumps(res))
