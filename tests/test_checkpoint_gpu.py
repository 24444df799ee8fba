"""Resume parity through the reference's checkpoint format: train two
steps, save_checkpoint, load into a fresh model + TrainStep, and the next step matches the
uninterrupted run bit for bit: the loss and every updated weight (same kernels, same moments, same
schedule position, and every gradient reduction summed in a fixed order)."""
import pytest
import torch

from test_model_gpu import load, mini_model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["noalign", "align"])
def test_resume_from_checkpoint(tag, tmp_path):
    from speech_transcript_embeddings_amd.checkpoint import load_checkpoint, save_checkpoint
    from speech_transcript_embeddings_amd.train import TrainStep, synthetic_batch
    meta, _ = load(tag)
    model = mini_model(meta)
    step = TrainStep(model, lr=1e-3, warmup=2, total_steps=10)
    data = synthetic_batch(2, 16000, 12, vocab=meta["mini"]["text"]["vocab_size"], seed=4)
    for s in range(2):
        torch.manual_seed(100 + s)
        step(*data)
    path = tmp_path / "best_model_gap.pt"
    save_checkpoint(path, model, step, epoch=0, train_metrics={"loss": float(step.last["loss"].item())},
                    val_metrics={}, temperature=0.1)
    fresh = mini_model(meta)
    step2 = TrainStep(fresh, lr=1e-3, warmup=2, total_steps=10)
    load_checkpoint(path, fresh, step2, map_location="cuda")
    assert step2.opt.t == 2 and step2.sched.step_count == 2
    torch.manual_seed(102)
    l1 = step(*data)
    torch.manual_seed(102)
    l2 = step2(*data)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)  # the forward is deterministic
    for (n, a), (_, b) in zip(model.state_dict().items(), fresh.state_dict().items()):
        assert torch.equal(a, b), (n, (a - b).abs().max().item())
