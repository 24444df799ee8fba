"""Which gradients differ between two identical TrainSteps (determinism diagnosis, GPU)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(align, spec, B=8):
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    torch.manual_seed(0)
    model = EnhancedAudioTextModel(use_word_alignment=align, text_layers_to_unfreeze=5, audio_layers_to_unfreeze=5,
                                   device="cuda", spec_augment=spec)
    model.audio_cfg.layerdrop = 0.0
    data = synthetic_batch(B, 160000, 64, device="cuda", seed=4)
    step = TrainStep(model, lr=0.0, warmup=1, total_steps=10, micro_batch=B, max_text_length=64)
    st = model.store
    if "--norefresh" in sys.argv:    # rebuild the cached Wᵀ lazily on the using stream instead
        st.refresh_transposes = lambda stream: None
    if "--refresh-main" in sys.argv:  # the refresh on the step's own stream
        r0 = st.refresh_transposes
        st.refresh_transposes = lambda stream: r0(torch.cuda.current_stream())
    if "--refresh-join" in sys.argv:  # the refresh on the side stream, then a full join
        r1 = st.refresh_transposes

        def rj(stream):
            r1(stream)
            if stream is not None:
                torch.cuda.current_stream().wait_stream(stream)
        st.refresh_transposes = rj
    gs = []
    eng = model.engine
    snaps = []
    ab0 = eng.audio_backward

    def ab(dh, ctx, layers_done=None):
        snaps[-1]["dah"] = dh.clone()
        return ab0(dh, ctx, layers_done)
    eng.audio_backward = ab
    cb0 = eng._conformer_bwd

    def cb(i, sv, dx5, *a, **k):
        snaps[-1][f"in{i}"] = None if dx5 is None else dx5.clone()
        for key in ("x", "x1", "x2", "x3", "x4", "qkv", "o", "o_lo", "lse", "z1", "z2", "pw1", "cv"):
            if sv.get(key) is not None:
                snaps[-1][f"sv{i}.{key}"] = sv[key].clone()
        r = cb0(i, sv, dx5, *a, **k)
        snaps[-1][f"out{i}"] = None if r[0] is None else r[0].clone()
        return r
    eng._conformer_bwd = cb
    busy = torch.cuda.Stream() if "--busy" in sys.argv else None
    if busy is not None:
        xa = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(2):
        snaps.append({})
        torch.manual_seed(123)
        np.random.seed(7)
        if busy is not None:   # unrelated work on another stream, queued to overlap the step
            busy.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(busy):
                for _k in range(60):
                    xa = (xa @ xa).clamp_(-1, 1)
        step(*data)
        torch.cuda.synchronize()
        gs.append(st.grad[: st.n_grad].clone())
    diffs = [k for k in snaps[0] if snaps[0][k] is not None and not torch.equal(snaps[0][k], snaps[1][k])]
    print("differing intermediates:", diffs[:40], flush=True)
    bad = []
    for sl in st.slots.values():
        if sl.segment not in ("enc", "head"):
            continue
        a, b = gs[0][sl.offset:sl.offset + sl.numel], gs[1][sl.offset:sl.offset + sl.numel]
        if not torch.equal(a, b):
            bad.append((sl.name, int((a != b).sum()), sl.numel, (a - b).abs().max().item()))
    print(f"args={sys.argv[1:]} align={align} spec={spec} text_stream={os.environ.get('STE_TEXT_STREAM', '1')}: {len(bad)} tensors differ",
          flush=True)
    for x in bad[:60]:
        print("   ", x, flush=True)


if __name__ == "__main__":
    run(align="--align" in sys.argv, spec="--spec" in sys.argv)
