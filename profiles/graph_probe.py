"""Does a HIP graph of the whole c2 training step pay?  Times (a) the eager step (Python + ctypes
launches, two streams), (b) its enqueue-only host time, (c) one captured hipGraph of the same step
replayed.  The replay repeats the captured step's per-step scalars (dropout seed, lr factor, Adam
step), which is fine for timing and nothing else.

    python profiles/graph_probe.py [--batch 64] [--steps 10] [--seconds 10]

A tiny batch (--batch 2 --seconds 1) makes the GPU work small, so the eager step time there is
the host's cost of issuing one step (≈ the same ~2,000 launches).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--seconds", type=float, default=10.0)
    a = ap.parse_args()
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    model = EnhancedAudioTextModel(text_layers_to_unfreeze=3, audio_layers_to_unfreeze=3, device="cuda",
                                   spec_augment=False)
    model.audio_cfg.layerdrop = 0.0
    step = TrainStep(model, warmup=100, total_steps=100000)
    d = synthetic_batch(a.batch, int(a.seconds * 16000), 64, device="cuda", seed=0)
    out = {}
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            step(*d)
        torch.cuda.synchronize()
        enq = []
        t0 = time.perf_counter()
        for _ in range(a.steps):
            t1 = time.perf_counter()
            step(*d)
            enq.append((time.perf_counter() - t1) * 1e3)
        torch.cuda.synchronize()
        out["eager_ms"] = round((time.perf_counter() - t0) / a.steps * 1e3, 3)
        out["eager_enqueue_ms"] = round(sorted(enq)[len(enq) // 2], 3)
    torch.cuda.synchronize()
    model.store._prebuilt = None       # no cross-capture event waits
    side = model.engine._side_stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(*d)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    model.store._prebuilt = None
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    out["graph_ms"] = round((time.perf_counter() - t0) / a.steps * 1e3, 3)
    out["loss"] = float(step.last["loss"].item())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
