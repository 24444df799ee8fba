"""Checkpoint format parity.

The reference saves `torch.save({...}, "best_model_loss.pt" / "best_model_gap.pt")` with the
keys of training/trainer_unfreeze.py:1617-1633 (model_state_dict from the module tree,
optimizer_state_dict from torch.optim.AdamW, metrics and the constructor arguments), and its
inference script restores `model.load_state_dict(checkpoint["model_state_dict"])` (strict,
inference.py:48-83).  `save_checkpoint` writes the same dict from this framework's model and
fused optimizer; `load_checkpoint` reads either side's files:

* model_state_dict: EnhancedAudioTextModel mirrors the reference's module tree name by name
  (tests/test_model_tree.py), so the state dict interchanges with `strict=True`;
* optimizer_state_dict: FusedAdamW.state_dict() is torch.optim.AdamW's layout with the
  reference's param-group numbering (ref:1486-1519), and FusedAdamW.load_state_dict() takes a
  reference AdamW's;
* files are read with torch.load(weights_only=True) only (no pickled code runs).  The
  reference's metrics are numpy float64 scalars; the numpy scalar reconstructors are
  allow-listed for that load, and save_checkpoint itself writes plain Python floats.
"""
from __future__ import annotations

import numpy as np
import torch

REF_KEYS = ("epoch", "model_state_dict", "optimizer_state_dict", "train_metrics", "val_metrics", "temperature",
            "projection_dim", "use_cross_modal", "use_attentive_pooling", "use_word_alignment", "freeze_encoders",
            "text_layers_to_unfreeze", "audio_layers_to_unfreeze")


def _plain(v):
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return type(v)(_plain(x) for x in v)
    if isinstance(v, np.generic):
        return v.item()
    return v


def checkpoint_dict(model, optimizer, *, epoch, train_metrics, val_metrics, temperature):
    """The reference's checkpoint dict (ref:1617-1633).  `optimizer` is a FusedAdamW, a
    TrainStep (its schedule-aware optimizer_state_dict()), or any object with state_dict()."""
    if hasattr(optimizer, "optimizer_state_dict"):
        osd = optimizer.optimizer_state_dict()
    else:
        osd = optimizer.state_dict()
    return {
        "epoch": epoch,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": osd,
        "train_metrics": _plain(train_metrics),
        "val_metrics": _plain(val_metrics),
        "temperature": temperature,
        "projection_dim": model.projection_dim,
        "use_cross_modal": model.use_cross_modal,
        "use_attentive_pooling": model.use_attentive_pooling,
        "use_word_alignment": model.use_word_alignment,
        "freeze_encoders": model.freeze_encoders,
        "text_layers_to_unfreeze": model.text_layers_to_unfreeze,
        "audio_layers_to_unfreeze": model.audio_layers_to_unfreeze,
    }


def save_checkpoint(path, model, optimizer, *, epoch, train_metrics, val_metrics, temperature):
    d = checkpoint_dict(model, optimizer, epoch=epoch, train_metrics=train_metrics, val_metrics=val_metrics,
                        temperature=temperature)
    torch.save(d, path)
    return d


def _safe_load(path, map_location):
    allow = [np.dtype, type(np.dtype(np.float64)), type(np.dtype(np.float32))]
    try:
        from numpy.core.multiarray import scalar as _np_scalar  # numpy < 2 name, still present in 2.x
    except ImportError:  # pragma: no cover
        from numpy._core.multiarray import scalar as _np_scalar
    allow.append(_np_scalar)
    with torch.serialization.safe_globals(allow):
        return torch.load(path, map_location=map_location, weights_only=True)


def load_checkpoint(path, model=None, optimizer=None, *, map_location=None, strict=True):
    """Read a checkpoint written by either framework.  Loads model_state_dict into `model`
    (strict by default, as inference.py does) and optimizer_state_dict into `optimizer` (a
    FusedAdamW or TrainStep) when given; returns the checkpoint dict."""
    ckpt = _safe_load(path, map_location if map_location is not None else "cpu")
    if optimizer is not None and hasattr(optimizer, "sync"):
        # an update still running on the optimizer's own stream (overlap_optimizer) writes the
        # master weights: the load below must come after it, not race it
        optimizer.sync()
    if model is not None:
        model.load_state_dict(ckpt["model_state_dict"], strict=strict)
    if optimizer is not None and "optimizer_state_dict" in ckpt:
        if hasattr(optimizer, "load_optimizer_state_dict"):
            optimizer.load_optimizer_state_dict(ckpt["optimizer_state_dict"])
        else:
            optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    return ckpt
