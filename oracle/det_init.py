"""ORACLE / test infrastructure — deterministic, portable parameter values.

Every parameter value is a pure function of (parameter name, shape, base seed)
through numpy's PCG64, so the reference model (when generating golden fixtures
in the survey container), the CPU oracle and the GPU model all load bit-identical
weights without shipping checkpoints.
"""
from __future__ import annotations

import zlib

import numpy as np


def param_value(name: str, shape, base_seed: int = 1234) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode()) ^ base_seed))
    shape = tuple(int(s) for s in shape)
    leaf = name.rsplit(".", 1)[-1]
    is_ln = ("norm" in name.lower() or "LayerNorm" in name) and leaf in ("weight", "bias")
    if is_ln and leaf == "weight":
        v = 1.0 + 0.1 * rng.standard_normal(shape)
    elif leaf == "bias" or name.endswith("in_proj_bias") or name.endswith("pos_bias_u") or name.endswith("pos_bias_v"):
        v = 0.05 * rng.standard_normal(shape)
    else:
        fan_in = shape[-1] if len(shape) >= 2 else max(shape[0], 1)
        if len(shape) == 3:  # conv1d [out, in/groups, k]
            fan_in = shape[1] * shape[2]
        std = min(0.08, 1.0 / np.sqrt(max(fan_in, 1)))
        v = std * rng.standard_normal(shape)
    return v.astype(np.float32)


def state_dict_values(named_shapes, base_seed: int = 1234) -> dict:
    return {n: param_value(n, s, base_seed) for n, s in named_shapes}


SAMPLE_K = 24


def sample_indices(name: str, numel: int, k: int = SAMPLE_K) -> np.ndarray:
    """Fixed flat indices used to record sampled gradient / update entries in fixtures."""
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(("idx:" + name).encode())))
    k = min(k, numel)
    return np.sort(rng.choice(numel, size=k, replace=False)).astype(np.int64)
