"""Golden vectors for the wav2vec2 raw-waveform audio encoder.

    python tests/golden/make_w2v2_golden.py      (CPU, this container; writes w2v2_golden.npz)

The reference hands raw samples to transformers' Wav2Vec2Model (ref:training/
trainer_unfreeze.py:587-641 -> tf:models/wav2vec2/modeling_wav2vec2.py:1244-1375); this script
runs THAT model (the in-container transformers) at mini dims in float64, training mode with every
dropout / layerdrop / SpecAugment probability 0, on seeded synthetic waveforms:
  * forward: last_hidden_state;
  * backward: the gradient of Σ(last_hidden_state · cot) w.r.t. every parameter (cot seeded).
Two cases: a ragged batch with a sample-level attention mask, and a batch without a mask (what
wav2vec2-base's processor returns).  LayerNorm / GroupNorm affines and all biases are
randomised so that each parameter's role is visible in the outputs.  Data only (inputs,
parameters, expected outputs) goes into the .npz.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent

MINI = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=1, intermediate_size=128,
            conv_dim=(64, 64, 64), conv_kernel=(10, 3, 2), conv_stride=(5, 2, 2), num_conv_pos_embeddings=16,
            num_conv_pos_embedding_groups=2, layer_norm_eps=1e-5, hidden_dropout=0.0, activation_dropout=0.0,
            attention_dropout=0.0, feat_proj_dropout=0.0, layerdrop=0.0, mask_time_prob=0.0,
            feat_extract_norm="group", conv_bias=False, do_stable_layer_norm=False)
CASES = {"mask": dict(B=3, N=4000, lengths=(4000, 3100, 2205)), "nomask": dict(B=2, N=3200, lengths=None)}


def build(seed=0):
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    torch.manual_seed(seed)
    cfg = Wav2Vec2Config(**MINI, attn_implementation="eager")
    m = Wav2Vec2Model(cfg)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            leaf = n.rsplit(".", 1)[-1]
            if ("layer_norm" in n) and leaf == "weight":
                p.copy_(1.0 + 0.2 * torch.randn(p.shape, generator=g))
            elif leaf == "bias":
                p.copy_(0.1 * torch.randn(p.shape, generator=g))
    return m.double().train()


def waves(case, seed):
    g = np.random.default_rng(seed)
    B, N = case["B"], case["N"]
    t = np.arange(N) / 16000.0
    x = np.zeros((B, N), np.float32)
    for b in range(B):
        f0 = 120 + 60 * b
        x[b] = (0.5 * np.sin(2 * np.pi * f0 * t) + 0.3 * np.sin(2 * np.pi * 3.1 * f0 * t)
                + 0.2 * g.standard_normal(N)).astype(np.float32)
    mask = None
    if case["lengths"] is not None:
        mask = np.zeros((B, N), np.int64)
        for b, L in enumerate(case["lengths"]):
            mask[b, :L] = 1
            x[b, L:] = 0.0
    return x, mask


def main():
    m = build()
    out = {}
    sd = {k: v.float().numpy() for k, v in m.state_dict().items()}
    for k, v in sd.items():
        out["param/" + k] = v
    for ci, (name, case) in enumerate(CASES.items()):
        x, mask = waves(case, 10 + ci)
        xt = torch.from_numpy(x).double()
        mt = None if mask is None else torch.from_numpy(mask)
        m.zero_grad(set_to_none=True)
        h = m(input_values=xt, attention_mask=mt).last_hidden_state
        g = torch.Generator().manual_seed(100 + ci)
        cot = torch.randn(h.shape, generator=g, dtype=torch.float64)
        (h * cot).sum().backward()
        out[f"{name}/wave"] = x
        if mask is not None:
            out[f"{name}/mask"] = mask
        out[f"{name}/hidden"] = h.detach().float().numpy()
        out[f"{name}/cot"] = cot.float().numpy()
        for n, p in m.named_parameters():
            if p.grad is not None:
                out[f"{name}/grad/{n}"] = p.grad.float().numpy()
    np.savez_compressed(HERE / "w2v2_golden.npz", **out)
    (HERE / "w2v2_golden.json").write_text(json.dumps({"config": MINI, "cases": CASES}, indent=1) + "\n")
    print("wrote", HERE / "w2v2_golden.npz", sum(v.size for v in out.values()), "values")


if __name__ == "__main__":
    main()
