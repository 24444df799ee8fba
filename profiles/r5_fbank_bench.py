"""Isolated ste_fbank at the c2 / c5 batch shapes (64 x 10 s, 16 x 30 s): HIP-event time per call."""
import json
import sys
import torch
sys.path.insert(0, ".")
from speech_transcript_embeddings_amd import ops

res = {}
for name, B, sec in (("c2", 64, 10.0), ("c5", 16, 30.0)):
    N = int(sec * 16000)
    wav = torch.randn(B, N, device="cuda") * 0.1
    lens = torch.full((B,), N, dtype=torch.int32, device="cuda")
    T = ((1 + (N - 400) // 160) + 1) // 2
    feats, mask = ops.fbank(wav, lens, T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        ops.fbank(wav, lens, T, feats=feats, mask=mask)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = 4 * B * N + feats.numel() * 4 + mask.numel() * 8
    res[name] = {"us": round(us, 2), "MB": round(nbytes / 1e6, 2), "frac_of_8TBps": round(nbytes / us / 8e6, 4)}
print(json.dumps(res))
