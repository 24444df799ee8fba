"""Isolated GLU + depthwise-conv backward (ste_glu_dwconv_bwd) with the weight gradient, at the c2
and c5 Conformer shapes: HIP-event time per call, and a checksum of the outputs (the A/B of a
numerics-neutral change must print identical sums)."""
import json
import sys
import torch
sys.path.insert(0, ".")
from speech_transcript_embeddings_amd import ops

res = {}
for name, B, T in (("c2", 64, 499), ("c5", 64, 1499)):
    C, K = 1024, 31
    torch.manual_seed(0)
    pre = torch.randn(B * T, 2 * C, device="cuda").bfloat16()
    w = torch.randn(C, K, device="cuda") * 0.1
    dout = torch.randn(B * T, C, device="cuda").bfloat16()
    dpre = torch.empty(B * T, 2 * C, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(C, K, device="cuda")
    ops.glu_dwconv_bwd(pre, w, dout, dpre, dw, B, T)
    chk = [float(dpre.float().sum()), float(dw.double().sum())]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        ops.glu_dwconv_bwd(pre, w, dout, dpre, dw, B, T)
    e1.record()
    torch.cuda.synchronize()
    res[name] = {"us": round(e0.elapsed_time(e1) * 1e3 / reps, 1), "checksum": chk}
print(json.dumps(res))
