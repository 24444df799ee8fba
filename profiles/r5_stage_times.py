"""Per-stage timeline of one training step at a per-GPU batch (c3's local 32 by default), for the
data-parallel all-reduce model of DESIGN §5.  One GPU, world size 1: GradSync's collectives do not
run, so the step is the N = 1 compute alone; this records, on the step's stream, HIP events at

  step start | backward start | each GradSync stage turning final (heads, audio_layers, audio,
  text: the points where a multi-GPU run starts that block's RCCL all-reduce) | backward end |
  optimizer end

and prints the mean offsets (ms) with the dense byte volume of every stage's all-reduce, as JSON.

    python profiles/r5_stage_times.py [--batch 32] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import GradSync, TrainStep, synthetic_batch

    model = EnhancedAudioTextModel(text_layers_to_unfreeze=3, audio_layers_to_unfreeze=3, device="cuda:0",
                                   spec_augment=False)
    model.audio_cfg.layerdrop = 0.0
    step = TrainStep(model, warmup=100, total_steps=100000, micro_batch=args.batch, max_text_length=64)
    data = synthetic_batch(args.batch, 160000, 64, device="cuda:0", seed=0)
    gs = step.gradsync
    marks = []

    def ev(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((name, e))

    orig_stage = gs.stage_done
    gs.stage_done = lambda stage, ids=None: (ev(stage), orig_stage(stage, ids))[1]
    eng = model.engine
    orig_bwd = eng.backward

    def bwd(*a, **k):
        ev("backward_start")
        r = orig_bwd(*a, **k)
        ev("backward_end")
        return r

    eng.backward = bwd
    stream = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    rows = []
    with torch.cuda.stream(stream):
        for it in range(args.warmup + args.steps):
            marks.clear()
            ev("step_start")
            step(*data)
            ev("step_end")
            torch.cuda.synchronize()
            if it >= args.warmup:
                t0 = marks[0][1]
                rows.append({n: t0.elapsed_time(e) for n, e in marks})
    keys = list(rows[0].keys())
    mean = {k: round(sum(r[k] for r in rows) / len(rows), 3) for k in keys}
    # dense all-reduce volume per stage (fp32 gradient bytes; the word table goes row-sparse)
    g = gs.store.grad
    vol = {}
    for stg in GradSync.STAGES:
        vol[stg] = sum(b - a for a, b in gs.ranges[stg]) * g.element_size()
    words = None
    if gs.words is not None:
        words = {"table_rows": gs.words.shape[0], "row_bytes": gs.words.shape[1] * 4,
                 "sparse_capacity_ids": gs.capacity}
    print(json.dumps({"batch": args.batch, "steps": args.steps, "offsets_ms": mean,
                      "stage_bytes": vol, "word_table": words,
                      "note": "offsets from step start on the step's stream; stage = point its gradients are final"}))


if __name__ == "__main__":
    main()
