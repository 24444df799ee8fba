"""Audio front end and batch collation of the hot path.

* ``SeamlessM4TFeatureExtractor`` — drop-in for the extractor the reference builds with
  ``AutoFeatureExtractor.from_pretrained("facebook/w2v-bert-2.0")`` (ref:training/
  trainer_unfreeze.py:1387-1388) and calls per clip at ref:856-866:
  ``fe(np.ndarray, sampling_rate=16000, return_tensors="pt") -> {"input_features": [1,T,160],
  "attention_mask": [1,T]}``.  The arithmetic (x·2^15, povey window, 512-point power
  spectrum, 80 kaldi mel bins, log, per-utterance CMVN, stride-2 stacking) is the fused
  ``ste_fbank`` HIP kernel; a list of clips is one batched launch padded to the longest clip
  with ``padding_value`` like the transformers extractor's default ``padding=True``.
* ``fbank`` — the batched on-GPU variant the training step uses: raw waveforms [B, Nmax]
  + lengths -> (input_values [B,Tmax,160], attention_mask_audio [B,Tmax]) with
  ``custom_collate_fn``'s semantics (zero padding, mask[i, :T_i] = 1, ref:898-908).
* ``custom_collate_fn`` — the reference's collate (ref:880-921) for host-side items, so a
  reference DataLoader pipeline plugs in unchanged.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.nn.utils.rnn import pad_sequence

from . import ops

SAMPLE_RATE = 16000
FRAME, HOP = 400, 160


def num_frames(n_samples: int) -> int:
    """Stacked feature frames T = ceil(F/2), F = 1 + (N - 400) // 160 fbank frames (0 if N < 400)."""
    f = 1 + (n_samples - FRAME) // HOP if n_samples >= FRAME else 0
    return (f + 1) // 2


def fbank(wav: torch.Tensor, lengths: torch.Tensor | None = None, *, pad_value: float = 1.0, Tmax: int | None = None):
    """Batched GPU fbank with collate semantics.  wav fp32 [B, Nmax] on the GPU; lengths int [B]
    (default: all Nmax).  Returns (input_values fp32 [B,Tmax,160], attention_mask_audio int64 [B,Tmax])."""
    if wav.dim() != 2 or wav.dtype != torch.float32 or not wav.is_cuda:
        raise ValueError("fbank expects a float32 [B, N] waveform tensor on the GPU")
    B, N = wav.shape
    if lengths is None:
        lengths = torch.full((B,), N, dtype=torch.int32, device=wav.device)
    lengths = lengths.to(device=wav.device, dtype=torch.int32)
    if Tmax is None:
        Tmax = num_frames(int(lengths.max().item()))
    wav = wav if wav.stride(1) == 1 else wav.contiguous()
    return ops.fbank(wav, lengths, max(Tmax, 1), pad_value=pad_value, mask_mode=0)


class SeamlessM4TFeatureExtractor:
    """w2v-bert-2.0's feature extractor (feature_size=80, num_mel_bins=80, padding_value=1.0,
    sampling_rate=16000, stride=2) on the HIP fbank kernel."""

    model_input_names = ["input_features", "attention_mask"]

    def __init__(self, feature_size=80, num_mel_bins=80, padding_value=1.0, sampling_rate=SAMPLE_RATE, stride=2,
                 device=None):
        if (feature_size, num_mel_bins, sampling_rate, stride) != (80, 80, SAMPLE_RATE, 2):
            raise ValueError("only the w2v-bert-2.0 front end (80 mel bins, 16 kHz, stride 2) is implemented")
        self.feature_size, self.num_mel_bins, self.stride = feature_size, num_mel_bins, stride
        self.padding_value, self.sampling_rate = float(padding_value), sampling_rate
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

    def __call__(self, raw_speech, sampling_rate=None, return_tensors="pt", return_attention_mask=True, **_):
        if sampling_rate is not None and sampling_rate != self.sampling_rate:
            raise ValueError(f"The model corresponding to this feature extractor was trained using a sampling rate of "
                             f"{self.sampling_rate}. Please make sure that the provided `raw_speech` input was sampled "
                             f"with {self.sampling_rate} and not {sampling_rate}.")
        if return_tensors not in ("pt", None):
            raise ValueError("return_tensors must be 'pt' (features stay on the GPU)")
        batched = isinstance(raw_speech, (list, tuple)) or (hasattr(raw_speech, "ndim") and raw_speech.ndim == 2)
        clips = list(raw_speech) if batched else [raw_speech]
        clips = [torch.as_tensor(np.asarray(c, dtype=np.float32) if not torch.is_tensor(c) else c,
                                 dtype=torch.float32).reshape(-1) for c in clips]
        if any(c.numel() == 0 for c in clips):
            raise ValueError("empty waveform")
        lens = [c.numel() for c in clips]
        N = max(lens)
        wav = torch.zeros(len(clips), N, dtype=torch.float32)
        for i, c in enumerate(clips):
            wav[i, : lens[i]] = c
        wav = wav.to(self.device, non_blocking=True)
        lengths = torch.tensor(lens, dtype=torch.int32, device=self.device)
        T = max(num_frames(n) for n in lens)
        feats, mask = ops.fbank(wav, lengths, max(T, 1), pad_value=self.padding_value, mask_mode=1)
        out = {"input_features": feats}
        if return_attention_mask:
            out["attention_mask"] = mask
        return out


def custom_collate_fn(batch):
    """ref:880-921: pad ids/masks with 0, zero-pad features to the longest clip, audio mask
    1 over each clip's frames (the extractor's mask is ignored), is_corrupted = zeros."""
    batch = [b for b in batch if b is not None]
    if not batch:
        return None
    out = {}
    for k in ("input_ids_pos", "attention_mask_pos", "input_ids_neg", "attention_mask_neg"):
        out[k] = pad_sequence([b[k] for b in batch], batch_first=True, padding_value=0)
    audios = [b["input_values"] for b in batch]
    B, max_t, feat = len(audios), max(a.size(0) for a in audios), audios[0].size(1)
    dev = audios[0].device
    padded = torch.zeros((B, max_t, feat), dtype=audios[0].dtype, device=dev)
    amask = torch.zeros((B, max_t), dtype=torch.long, device=dev)
    for i, a in enumerate(audios):
        padded[i, : a.size(0)] = a
        amask[i, : a.size(0)] = 1
    out["input_values"] = padded
    out["attention_mask_audio"] = amask
    out["is_corrupted"] = torch.zeros(B, dtype=torch.long, device=dev)
    # host list of each clip's frames (not a tensor: the reference's loop moves tensors only), so
    # SpecAugment's span sampling needs no device->host sync once the mask is on the GPU
    out["audio_lengths"] = [int(a.size(0)) for a in audios]
    return out
