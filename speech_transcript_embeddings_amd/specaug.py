"""SpecAugment time masking of the audio encoder (w2v-bert training mode).

Mirrors transformers' Wav2Vec2BertModel._mask_hidden_states (time axis) and
_compute_mask_indices (tf:models/wav2vec2_bert/modeling_wav2vec2_bert.py:800-919, 944-988;
transformers 4.50.2 as pinned by the reference, same code in the 5.x here), which the
reference runs whenever the audio encoder is in training mode and config.mask_time_prob > 0
(w2v-bert-2.0: 0.05, spans of 10 frames, at least 2 spans).  The span sampling is host-side
numpy on the global RNG with the same sequence of draws as transformers, so a seeded run
masks exactly the frames the reference masks; the masked rows are then overwritten with
masked_spec_embed on the GPU (ste_spec_mask_fwd) and the backward routes their gradient into
masked_spec_embed (ste_spec_mask_bwd).
"""
from __future__ import annotations

import numpy as np
import torch


def compute_mask_indices(shape, mask_prob: float, mask_length: int, input_lengths=None, min_masks: int = 0):
    """bool [batch, seq] span mask; input_lengths = the valid frames of each row (the
    attention mask's row sums), None = all frames valid."""
    batch, seq = shape
    if mask_length < 1:
        raise ValueError("`mask_length` has to be bigger than 0.")
    if mask_length > seq:
        raise ValueError(f"`mask_length` has to be smaller than `sequence_length`, but got `mask_length`: "
                         f"{mask_length} and `sequence_length`: {seq}`")
    eps = np.random.rand(1).item()  # probabilistic rounding of the span count

    def n_spans(length):
        n = max(int(mask_prob * length / mask_length + eps), min_masks)
        if n * mask_length > seq:
            n = seq // mask_length
        if length - (mask_length - 1) < n:
            n = max(length - (mask_length - 1), 0)
        return n

    lengths = list(input_lengths) if input_lengths is not None else [seq] * batch
    mask = np.zeros((batch, seq), dtype=bool)
    n_max = n_spans(seq)
    if n_max == 0:
        return mask
    starts = []
    for length in lengths:
        n = n_spans(length)
        idx = np.random.choice(np.arange(length - (mask_length - 1)), n, replace=False)
        pad = idx[0] if len(idx) else seq - 1  # padding spans repeat the first start (or the last frame)
        starts.append(np.concatenate([idx, np.ones(n_max - n, dtype=np.int32) * pad]))
    starts = np.array(starts)
    spans = (starts[:, :, None] + np.arange(mask_length)[None, None, :]).reshape(batch, n_max * mask_length)
    spans = np.minimum(spans, seq - 1)
    np.put_along_axis(mask, spans, 1, -1)
    return mask


def upload_mask(sm, device):
    """bool [B, T] host mask -> int32 [B*T] on `device` through pinned memory, without blocking
    the host on the device queue (the caching host allocator keeps the pinned block alive until
    the copy has run)."""
    host = torch.from_numpy(np.ascontiguousarray(sm, dtype=np.int32).reshape(-1))
    if torch.device(device).type != "cuda":
        return host.to(device)
    return host.pin_memory().to(device, non_blocking=True)
