"""Isolated clip + AdamW (ste_adamw) over 150 M parameters (c2's trained set): HIP-event time per
launch, achieved GB/s at 30 B/param, and a checksum (A/B variants must agree bit for bit)."""
import json
import sys
import torch
sys.path.insert(0, ".")
from speech_transcript_embeddings_amd import ops

n = 150_000_000
torch.manual_seed(0)
p = torch.randn(n, device="cuda")
g = torch.randn(n, device="cuda") * 1e-3
m = torch.zeros(n, device="cuda")
v = torch.zeros(n, device="cuda")
pb = torch.empty(n, device="cuda", dtype=torch.bfloat16)
acc = torch.zeros(1, device="cuda", dtype=torch.float64)
ops.sumsq(g, acc)
kw = dict(lr=1e-5, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.01, step=1, sumsq_acc=acc, max_norm=1.0)
for _ in range(3):
    ops.adamw(p, g, m, v, pb, **kw)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 10
e0.record()
for _ in range(reps):
    ops.adamw(p, g, m, v, pb, **kw)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
print(json.dumps({"us": round(us, 1), "GBps": round(30 * n / us / 1e3, 1),
                  "checksum": [float(p.double().sum()), float(m.double().sum()), float(v.double().sum())]}))
