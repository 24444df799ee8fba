"""ORACLE — test infrastructure, NOT product code.

numpy restatement of the w2v-bert feature extractor arithmetic the reference
calls (ref:training/trainer_unfreeze.py:856-866 -> SeamlessM4TFeatureExtractor):
  tf:models/seamless_m4t/feature_extraction_seamless_m4t.py:112-138 (_extract_fbank_features),
  :240-301 (__call__: per-mel-bin CMVN ddof=1, pad to even frames, stride-2 stack, mask),
  tf:audio_utils.py:809-1017 (spectrogram), :638-729 (mel_filter_bank, kaldi scale,
  triangularize_in_mel_space), :786-787 (povey window).
Pinned by tests/golden/fbank_golden.npz generated from the reference's extractor
(tests/golden/make_golden.py).  Vectorised over frames (the reference loops in
Python per frame, tf:audio_utils.py:973-989); float64 spectra like the reference.
"""
from __future__ import annotations

import numpy as np

SR = 16000
FRAME = 400
HOP = 160
NFFT = 512
NMEL = 80
PREEMPH = 0.97
MEL_FLOOR = 1.192092955078125e-07


def _hz_to_mel_kaldi(f):
    return 1127.0 * np.log(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_filters() -> np.ndarray:
    """[257, 80] kaldi-scale triangular filters built in mel space, 20 Hz..8 kHz, no norm."""
    mel_min, mel_max = _hz_to_mel_kaldi(20.0), _hz_to_mel_kaldi(SR // 2)
    mel_freqs = np.linspace(mel_min, mel_max, NMEL + 2)
    fft_freqs = _hz_to_mel_kaldi((SR / ((257 - 1) * 2)) * np.arange(257))
    fdiff = np.diff(mel_freqs)
    slopes = mel_freqs[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / fdiff[:-1]
    up = slopes[:, 2:] / fdiff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def povey_window() -> np.ndarray:
    return np.power(np.hanning(FRAME), 0.85)  # symmetric (periodic=False)


def logmel(wave: np.ndarray) -> np.ndarray:
    """[F, 80] float32 log-mel of one clip (before CMVN)."""
    x = np.asarray(wave, dtype=np.float32).reshape(-1).astype(np.float64) * 32768.0
    nfr = 1 + (x.size - FRAME) // HOP
    idx = np.arange(FRAME)[None, :] + HOP * np.arange(nfr)[:, None]
    fr = x[idx]
    fr = fr - fr.mean(axis=1, keepdims=True)
    fr[:, 1:] = fr[:, 1:] - PREEMPH * fr[:, :-1]
    fr[:, 0] *= 1.0 - PREEMPH
    fr = fr * povey_window()[None, :]
    spec = np.fft.rfft(fr, n=NFFT, axis=1).astype(np.complex64)
    power = np.abs(spec, dtype=np.float64) ** 2
    mel = np.maximum(MEL_FLOOR, power @ mel_filters())
    return np.log(mel).astype(np.float32)


def extract(wave: np.ndarray, padding_value: float = 1.0):
    """One clip -> (input_features [T,160] float32, attention_mask [T] int64), extractor semantics."""
    f = logmel(wave)
    mean = f.mean(0, keepdims=True)
    var = f.var(0, ddof=1, keepdims=True)
    f = (f - mean) / np.sqrt(var + 1e-7)
    F_ = f.shape[0]
    mask = np.ones(F_, dtype=np.int64)
    if F_ % 2:
        f = np.concatenate([f, np.full((1, NMEL), padding_value, np.float32)], 0)
        mask = np.concatenate([mask, np.zeros(1, np.int64)])
    T = f.shape[0] // 2
    feats = f.reshape(T, 2 * NMEL).astype(np.float32)
    m = mask[np.arange(2 * T) % 2 == 1]
    return feats, m


def collate(items):
    """ref:880-921 audio part: zero-pad to Tmax; mask = 1 for t < T_i (extractor mask ignored)."""
    T = max(a.shape[0] for a in items)
    out = np.zeros((len(items), T, 2 * NMEL), np.float32)
    mask = np.zeros((len(items), T), np.int64)
    for i, a in enumerate(items):
        out[i, : a.shape[0]] = a
        mask[i, : a.shape[0]] = 1
    return out, mask


def num_stacked_frames(n_samples: int) -> int:
    F_ = 1 + (n_samples - FRAME) // HOP
    return (F_ + 1) // 2


def synth_wave(seed: int, n: int) -> np.ndarray:
    """SURVEY §8d synthetic clip: 0.1·N(0,1) + 3 sinusoids (100-3000 Hz, amp 0.05), clipped."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / SR
    x = 0.1 * rng.standard_normal(n)
    for f in rng.uniform(100, 3000, size=3):
        x += 0.05 * np.sin(2 * np.pi * f * t)
    return np.clip(x, -1, 1).astype(np.float32)
