"""Config-size fbank cases (BASELINE c2 / c5 clip lengths and the extractor's edge paths).

The waveforms are rebuilt from seeds here (oracle/fbank_ref.synth_wave, SURVEY §8d signal), so
tests/golden/fbank_golden_long.npz holds only the reference extractor's outputs for them:
  10s         c2-c4 clip (160,000 samples, T = 499)
  30s         c5 clip (480,000 samples, T = 1499)
  10s_oddF    160,160 samples: F = 999 fbank frames, odd -> the extractor pads one frame
  10s_edge    2 s of exact zeros (log-floor path) inside a loud clip scaled x8, clipped to +-4
  silence     1 s of zeros: every frame at the log floor, CMVN variance 0
"""
import numpy as np

LONG_CASES = (("10s", 1100, 160000), ("30s", 1101, 480000), ("10s_oddF", 1103, 160160),
              ("10s_edge", 1102, 160000), ("silence", 0, 16000))


def long_case_wave(name: str) -> np.ndarray:
    from oracle import fbank_ref
    seed, n = {c: (s, k) for c, s, k in LONG_CASES}[name]
    if name == "silence":
        return np.zeros(n, np.float32)
    w = fbank_ref.synth_wave(seed, n)
    if name == "10s_edge":
        w = np.clip(w * 8.0, -4.0, 4.0).astype(np.float32)
        w[32000:64000] = 0.0
    return w
