"""Diagnose TrainStep(overlap_optimizer=True) vs serial: which slots of master / grad differ,
with and without a sync between steps."""
import sys
import torch
from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch

B, N, L = 4, 64000, 32


def run(overlap, sync_each, nsteps=3):
    torch.manual_seed(0)
    model = EnhancedAudioTextModel(use_word_alignment=True, text_layers_to_unfreeze=3, audio_layers_to_unfreeze=3,
                                   device="cuda", spec_augment=False)
    model.audio_cfg.layerdrop = 0.0
    step = TrainStep(model, lr=1e-3, warmup=1, total_steps=10, micro_batch=B, max_text_length=L,
                     overlap_optimizer=overlap)
    batches = [synthetic_batch(B, N, L, device="cuda", seed=10 + i) for i in range(nsteps)]
    torch.cuda.synchronize()
    snaps = []
    for i in range(nsteps):
        torch.manual_seed(100 + i)
        loss = step(*batches[i]).clone()
        if sync_each:
            step.sync()
            torch.cuda.synchronize()
            st = model.store
            snaps.append((loss, st.grad[: st.n_grad].clone(), st.master.clone()))
        else:
            snaps.append((loss, None, None))
    step.sync()
    torch.cuda.synchronize()
    st = model.store
    return model, snaps, (st.grad[: st.n_grad].clone(), st.master.clone())


def where(st, diff):
    return sorted({sl.name for sl in st.slots.values() if diff[sl.offset:sl.offset + sl.numel].any()})


m0, s0, f0 = run(False, True)
for tag, ov, se in (("serial-nosync", False, False), ("overlap-sync", True, True), ("overlap-nosync", True, False)):
    m1, s1, f1 = run(ov, se)
    st = m1.store
    print(tag, "losses", [float(a[0]) for a in s1], "ref", [float(a[0]) for a in s0])
    for i in range(3):
        if s1[i][1] is not None:
            dg = s0[i][1] != s1[i][1]
            dm = s0[i][2] != s1[i][2]
            print(f"  step {i}: grad diff {int(dg.sum())} in {where(st, dg)[:8]}; master diff {int(dm.sum())} in {where(st, dm)[:8]}")
    dg = f0[0] != f1[0]
    dm = f0[1] != f1[1]
    print(f"  final: grad diff {int(dg.sum())} in {where(st, dg)[:8]}; master diff {int(dm.sum())} in {where(st, dm)[:8]}")
    sys.stdout.flush()
