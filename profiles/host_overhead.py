"""Host launch cost of one c2 training step vs its GPU time: is the CPU side (Python + ctypes
launches) ever the limiter?  Enqueue time = wall time of the step() call with the GPU idle at
its start (no synchronisation inside the step); GPU time = synchronised wall time per step.

    python profiles/host_overhead.py [--batch 64] [--steps 5]
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
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    model = EnhancedAudioTextModel(text_layers_to_unfreeze=3, audio_layers_to_unfreeze=3, device="cuda",
                                   spec_augment=False)
    model.audio_cfg.layerdrop = 0.0
    step = TrainStep(model, warmup=100, total_steps=100000)
    d = synthetic_batch(a.batch, 160000, 64, device="cuda", seed=0)
    for _ in range(3):
        step(*d)
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step(*d)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    print(json.dumps({"enqueue_ms": [round(x, 2) for x in enq], "step_ms": [round(x, 2) for x in tot]}), flush=True)


if __name__ == "__main__":
    main()
