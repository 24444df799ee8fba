"""Run-to-run determinism of the training step (checkpoint resume,
ref:training/trainer_unfreeze.py:1613-1678, is then bitwise).

Every cross-block reduction of the backward is ordered: GEMM bias gradients (per-wave partial
rows + ste_rowsum_ordered), ste_colsum, the LayerNorm column sums, the depthwise-conv weight
gradient, the attentive-pooling scorer bias, the SpecAugment embedding, the word / position
table rows (one writer per row, rows summed in token order), the token-type row and the
clip-norm Σg².  So the same step on the same weights, inputs and seeds gives bit-identical
gradients, clip norm and loss.

Workload: full w2v-bert-2.0 + XLM-R dims, B = 8 clips of 10 s (31,936 / 8 = 3,992 frame rows:
the Conformer dz GEMMs run on the 8-phase kernel with its column-sum epilogue), 64-token
transcripts, config-4 shape (5 + 5 unfrozen, alignment head), train mode with dropout and
SpecAugment on (seeded), one TrainStep at lr 0 (weights unchanged), repeated.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_train_step_bitwise_reproducible():
    from speech_transcript_embeddings_amd import ops
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    assert not ops.ATOMIC_SUMS
    torch.manual_seed(0)
    model = EnhancedAudioTextModel(use_word_alignment=True, text_layers_to_unfreeze=5, audio_layers_to_unfreeze=5,
                                   device="cuda", spec_augment=True)
    model.audio_cfg.layerdrop = 0.0
    B, N, L = 8, 160000, 64
    data = synthetic_batch(B, N, L, device="cuda", seed=4)
    step = TrainStep(model, lr=0.0, warmup=1, total_steps=10, micro_batch=B, max_text_length=L)
    st = model.store
    runs = []
    for _ in range(2):
        torch.manual_seed(123)
        np.random.seed(7)
        loss = step(*data)
        torch.cuda.synchronize()
        runs.append((loss.clone(), st.grad[: st.n_grad].clone(), step.opt.sumsq.clone(), st.master.clone()))
    (l0, g0, s0, m0), (l1, g1, s1, m1) = runs
    assert torch.equal(m0, m1)                   # lr 0: the weights did not move between the runs
    assert torch.equal(l0, l1), (l0.item(), l1.item())
    diff = (g0 != g1)
    if diff.any():
        bad = sorted({sl.name for sl in st.slots.values() if sl.segment in ("enc", "head")
                      and diff[sl.offset:sl.offset + sl.numel].any()})
        pytest.fail(f"{int(diff.sum())} gradient entries differ between identical steps, in {bad[:12]}")
    assert torch.equal(s0, s1)                   # clip_grad_norm_'s Σg², hence the clip coefficient
    assert float(g0.abs().sum()) > 0


@pytest.mark.timeout(600)
def test_overlapped_optimizer_bitwise_equal():
    """TrainStep(overlap_optimizer=True): clip + AdamW on their own stream, split into the blocks
    the next forward reads in order, each awaited right before its first read.  Three steps at a
    real learning rate (each step's forward reads the previous update) give bit-identical
    weights, moments, losses and gradients to the serial optimizer — a missed wait would read a
    half-updated weight or zero a gradient AdamW has not read yet."""
    from speech_transcript_embeddings_amd.model import EnhancedAudioTextModel
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    B, N, L = 4, 64000, 32
    out = []
    for overlap in (False, True):
        torch.manual_seed(0)
        model = EnhancedAudioTextModel(use_word_alignment=True, text_layers_to_unfreeze=3, audio_layers_to_unfreeze=3,
                                       device="cuda", spec_augment=False)
        model.audio_cfg.layerdrop = 0.0
        step = TrainStep(model, lr=1e-3, warmup=1, total_steps=10, micro_batch=B, max_text_length=L,
                         overlap_optimizer=overlap)
        batches = [synthetic_batch(B, N, L, device="cuda", seed=10 + i) for i in range(3)]
        torch.cuda.synchronize()
        losses = []
        for i in range(3):                     # back to back: step i+1's forward overlaps step i's AdamW
            torch.manual_seed(100 + i)
            losses.append(step(*batches[i]).clone())
        # read straight after the step, without step.sync(): total_norm() itself must wait for the
        # optimizer stream's Σg²
        tnorm = step.opt.total_norm()
        step.sync()
        torch.cuda.synchronize()
        st = model.store
        out.append((torch.stack(losses), st.grad[: st.n_grad].clone(), st.master.clone(), step.opt.exp_avg.clone(),
                    step.opt.exp_avg_sq.clone(), st.shadow.clone(), tnorm))
    (l0, g0, m0, a0, v0, s0, n0), (l1, g1, m1, a1, v1, s1, n1) = out
    assert torch.equal(l0, l1), (l0.tolist(), l1.tolist())
    assert n0 == n1 and n0 > 0, (n0, n1)
    assert torch.equal(g0, g1)
    assert torch.equal(m0, m1) and torch.equal(a0, a1) and torch.equal(v0, v1) and torch.equal(s0, s1)
    assert float((a0 != 0).sum()) > 0
