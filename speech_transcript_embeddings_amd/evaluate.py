"""Forward-only evaluation on the HIP path.

Mirrors the reference's validation loop and its metric helper:
  evaluate(model, data_loader, loss_fn, device, epoch=None, split="Validation", fp16=False)
      -> (metrics dict, all_similarities)           training/trainer_unfreeze.py:1165-1284
  to_human_readable(cosine, temperature=0.1, scale="prob")           trainer_unfreeze.py:924-939

Same names, arguments, metric keys and return values.  What differs is how a batch runs:
`EvalStep` computes the three embeddings with no saved activations (engine.forward(save=False):
each encoder layer's buffers go back to the allocator as the next layer runs, and the FFN GEMMs
skip the pre-activation copies only backward reads), then S = A·[Tp;Tn]ᵀ on the fp32 MFMA
similarity kernel and s_pos, s_neg and the AlignmentAwareInfoNCE value on the pair-loss kernel,
the same kernels the training step uses.  Per-batch results stay on the device and the metrics
are reduced once at the end, so the loop never waits on the host inside a batch (the
reference's per-batch `.item()` / `.cpu()` calls each synchronise).
"""
from __future__ import annotations

import logging

import numpy as np
import torch

from . import ops
from .model import AlignmentAwareInfoNCE, EnhancedAudioTextModel

logger = logging.getLogger(__name__)
F32 = torch.float32
_BATCH_KEYS = ("input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg", "input_values",
               "attention_mask_audio")


def to_human_readable(cosine: torch.Tensor, temperature: float = 0.1, scale: str = "prob") -> torch.Tensor:
    """ref:924-939.  "0to1": (cos + 1) / 2;  "prob": sigmoid(cos / τ)."""
    if scale == "0to1":
        return (cosine + 1.) * 0.5
    elif scale == "prob":
        return torch.sigmoid(cosine / temperature)
    else:
        raise ValueError(f"Unknown scale '{scale}'. Use '0to1' or 'prob'.")


class EvalStep:
    """One forward-only pass over a batch -> (s_pos [b], s_neg [b], loss [1]) device tensors.

    s_pos[i] = <a_i, tp_i> and s_neg[i] = <a_i, tn_i> of the L2-normalised embeddings (ref:1196-
    1197), loss = AlignmentAwareInfoNCE(τ, alignment_weight, corrupt_gamma)(s_pos, s_neg,
    last_alignment_scores) (ref:1203).  The model's train/eval mode is the caller's (evaluate()
    sets eval, as the reference does)."""

    def __init__(self, model: EnhancedAudioTextModel, temperature=0.1, alignment_weight=0.3, corrupt_gamma=0.35):
        self.model = model
        self.tau, self.aw, self.gamma = float(temperature), float(alignment_weight), float(corrupt_gamma)

    @torch.no_grad()
    def __call__(self, batch):
        m = self.model
        for k in _BATCH_KEYS:
            if batch[k].device.type != "cuda":
                raise RuntimeError(f"batch[{k!r}] must be on the GPU (libste.so has no CPU path)")
        m.store.sync_shadow()
        tf_p, tf_n, af, align, _ = m.engine.forward(batch, m.training, save=False)
        m.last_alignment_scores = align if m.use_word_alignment else None
        B, P = af.shape
        dev = af.device
        tn_all = torch.empty(2 * B, P, device=dev, dtype=F32)
        an = torch.empty(B, P, device=dev, dtype=F32)
        nrm = torch.empty(3 * B, device=dev, dtype=F32)
        ops.l2norm_fwd(tf_p.contiguous(), tn_all[:B], nrm[:B])
        ops.l2norm_fwd(tf_n.contiguous(), tn_all[B:], nrm[B:2 * B])
        ops.l2norm_fwd(af.contiguous(), an, nrm[2 * B:])
        S = torch.empty(B, 2 * B, device=dev, dtype=F32)
        ops.similarity(an, tn_all, S)
        sp, sn, loss = (torch.empty(n, device=dev, dtype=F32) for n in (B, B, 1))
        al = align.contiguous().float() if align is not None else None
        L = al.shape[1] if al is not None else 0
        ops.pair_loss_fwd(S, B, al, B, L, self.tau, self.aw, self.gamma, sp, sn, loss)
        return sp, sn, loss


def evaluate(model, data_loader, loss_fn, device, epoch: int = None, split: str = "Validation", fp16: bool = False):
    """ref:1165-1284.  Returns (metrics, all_similarities) with the reference's keys: loss,
    avg_similarity, median_similarity, std_similarity, clean_similarity, corrupt_similarity,
    similarity_gap; all_similarities = sigmoid(s_pos/0.1) per sample.  A batch that raises is
    logged and skipped, as in the reference.  `fp16` is accepted for signature parity: the HIP
    path always runs bf16 MFMA operands with fp32 accumulation."""
    model.eval()
    if isinstance(loss_fn, AlignmentAwareInfoNCE):
        step = EvalStep(model, loss_fn.temperature, loss_fn.alignment_weight, loss_fn.corrupt_gamma)
        native_loss = True
    else:  # any other loss callable gets (s_pos, s_neg, alignment_scores=...) like the reference
        step = EvalStep(model)
        native_loss = False
    s_pos_all, s_neg_all, loss_sum = [], [], []
    sample_count = 0
    desc = f"Epoch {epoch} [{split}]" if epoch is not None else f"[{split}]"
    with torch.no_grad():
        for batch_idx, batch in enumerate(data_loader):
            try:
                if batch is None:
                    logger.warning("Skipping None batch during evaluation")
                    continue
                batch = {k: v.to(device, non_blocking=True) if isinstance(v, torch.Tensor) else v
                         for k, v in batch.items()}
                sp, sn, loss = step(batch)
                if not native_loss:
                    loss = loss_fn(sp, sn, alignment_scores=getattr(model, "last_alignment_scores", None))
                    loss = loss.reshape(1).float()
                bsz = sp.shape[0]
                s_pos_all.append(sp)
                s_neg_all.append(sn)
                loss_sum.append(loss * bsz)
                sample_count += bsz
            except Exception as e:  # the reference logs and continues (ref:1253-1258)
                logger.error(f"Error in evaluation batch {batch_idx}: {e}")
                logger.error(f"Batch keys: {list(batch.keys() if batch else [])}")
                import traceback
                logger.error(traceback.format_exc())
                continue
    if sample_count == 0:
        logger.warning(f"No valid samples were processed during {split} evaluation")
        return {k: 0.0 for k in ("loss", "avg_similarity", "median_similarity", "std_similarity", "clean_similarity",
                                  "corrupt_similarity", "similarity_gap")}, []
    # one device->host transfer for the whole split
    clean = to_human_readable(torch.cat(s_pos_all), temperature=0.1, scale="prob").cpu().numpy()
    corrupt = to_human_readable(torch.cat(s_neg_all), temperature=0.1, scale="prob").cpu().numpy()
    total_loss = float(torch.cat(loss_sum).sum().item())
    all_similarities = list(clean)
    avg_similarity = np.mean(all_similarities)
    std_similarity = np.std(all_similarities)
    median_similarity = np.median(all_similarities)
    avg_clean = np.mean(clean)
    avg_corrupt = np.mean(corrupt)
    similarity_gap = avg_clean - avg_corrupt
    logger.info(f"{desc} {split} metrics:")
    logger.info(f"  Loss: {total_loss / sample_count:.4f}")
    logger.info(f"  Average similarity: {avg_similarity:.4f}")
    logger.info(f"  Median similarity: {median_similarity:.4f}")
    logger.info(f"  Clean sample similarity: {avg_clean:.4f}")
    logger.info(f"  Corrupted sample similarity: {avg_corrupt:.4f}")
    logger.info(f"  Similarity gap (clean - corrupt): {similarity_gap:.4f}")
    metrics = {
        "loss": total_loss / sample_count,
        "avg_similarity": avg_similarity,
        "median_similarity": median_similarity,
        "std_similarity": std_similarity,
        "clean_similarity": avg_clean,
        "corrupt_similarity": avg_corrupt,
        "similarity_gap": similarity_gap,
    }
    return metrics, all_similarities
