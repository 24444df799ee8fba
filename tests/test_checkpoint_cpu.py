"""Checkpoint format parity (ref training/trainer_unfreeze.py:1617-1633,
inference.py:48-83) on the CPU: no kernel runs, only the format.

* FusedAdamW.state_dict() is torch.optim.AdamW's layout with the reference's param-group
  numbering (ref:1486-1519): a reference AdamW built the reference's way loads it, and its
  state_dict (after a real torch step) loads back into FusedAdamW with every moment in place;
* the checkpoint dict carries exactly the reference's keys, survives torch.save /
  torch.load(weights_only=True), and its model_state_dict loads strictly into a fresh model;
* a reference-style file whose metrics are numpy float64 scalars loads with the safe loader."""
import numpy as np
import pytest
import torch

from test_model_gpu import load, mini_model


def _model(tag="noalign", **kw):
    meta, _ = load(tag)
    m = mini_model(meta, device="cpu", **kw)
    return m


def _ref_adamw(model, lr=2.1e-3, partial=True):
    """The reference's optimizer construction (ref:1486-1519)."""
    if partial:
        enc, rest = [], []
        for n, p in model.named_parameters():
            if p.requires_grad:
                (enc if ("text_encoder" in n or "audio_encoder" in n) else rest).append(p)
        return torch.optim.AdamW([{"params": enc, "lr": lr / 50, "weight_decay": 0.01},
                                  {"params": rest, "lr": lr, "weight_decay": 0.01}])
    return torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=lr, weight_decay=0.01)


def _filled_opt(model):
    from speech_transcript_embeddings_amd.train import FusedAdamW
    opt = FusedAdamW(model)
    g = torch.Generator().manual_seed(1)
    opt.exp_avg.copy_(torch.randn(opt.exp_avg.shape, generator=g))
    opt.exp_avg_sq.copy_(torch.rand(opt.exp_avg_sq.shape, generator=g))
    opt.t = 3
    opt.last_factor = 0.5
    return opt


@pytest.mark.parametrize("tag", ["noalign", "align"])
def test_fused_adamw_state_dict_loads_into_reference_adamw(tag):
    model = _model(tag)
    opt = _filled_opt(model)
    sd = opt.state_dict()
    ref = _ref_adamw(model)
    ref.load_state_dict(sd)  # torch validates group sizes and keys
    st = model.store
    params = dict(model.named_parameters())
    n_state = 0
    for n, p in params.items():
        s = st.slots[n]
        if s.segment not in ("enc", "head"):
            assert p not in ref.state or not ref.state[p]
            continue
        rs = ref.state[p]
        sl = slice(s.offset, s.offset + s.numel)
        assert torch.equal(rs["exp_avg"], opt.exp_avg[sl].view(s.shape))
        assert torch.equal(rs["exp_avg_sq"], opt.exp_avg_sq[sl].view(s.shape))
        assert float(rs["step"]) == 3.0
        n_state += 1
    assert n_state > 0
    for g, base in zip(ref.param_groups, (2.1e-3 / 50, 2.1e-3)):
        assert g["initial_lr"] == pytest.approx(base) and g["lr"] == pytest.approx(0.5 * base)
    # same group keys as a real torch AdamW after a LambdaLR-scheduled step
    real = _ref_adamw(_model(tag))
    torch.optim.lr_scheduler.LambdaLR(real, lambda s: 1.0)
    assert [set(g) for g in real.state_dict()["param_groups"]] == [set(g) for g in sd["param_groups"]]


def test_reference_adamw_state_loads_into_fused_adamw():
    model = _model()
    ref = _ref_adamw(model)
    sched = torch.optim.lr_scheduler.LambdaLR(ref, lambda s: (s + 1) / 4)
    g = torch.Generator().manual_seed(2)
    for n, p in model.named_parameters():  # what a reference step leaves: the pooler (unused) and
        if model.store.slots[n].segment in ("enc", "head"):  # masked_spec_embed get no gradient
            p.grad = torch.randn(p.shape, generator=g)
    with torch.no_grad():
        before = {n: p.detach().clone() for n, p in model.named_parameters()}
    ref.step()
    sched.step()
    ref.step()
    sched.step()
    sd = ref.state_dict()
    with torch.no_grad():  # the moments are what is checked; put the weights back
        for n, p in model.named_parameters():
            p.copy_(before[n])
    from speech_transcript_embeddings_amd.train import FusedAdamW
    opt = FusedAdamW(model)
    opt.load_state_dict(sd)
    assert opt.t == 2
    st = model.store
    for n, p in model.named_parameters():
        s = st.slots[n]
        if s.segment not in ("enc", "head"):
            continue
        sl = slice(s.offset, s.offset + s.numel)
        assert torch.equal(opt.exp_avg[sl].view(s.shape), ref.state[p]["exp_avg"]), n
        assert torch.equal(opt.exp_avg_sq[sl].view(s.shape), ref.state[p]["exp_avg_sq"]), n
    assert opt.groups[0]["lr"] == pytest.approx(2.1e-3 / 50) and opt.groups[1]["lr"] == pytest.approx(2.1e-3)
    assert opt.last_factor == pytest.approx(3 / 4)
    # and back: the reloaded state reproduces the reference's state_dict values
    sd2 = opt.state_dict()
    for i, ps in sd["state"].items():
        assert torch.equal(sd2["state"][i]["exp_avg"], ps["exp_avg"])
    with pytest.raises(ValueError):
        bad = {"state": {}, "param_groups": sd["param_groups"][:1]}
        opt.load_state_dict(bad)


def test_single_group_when_not_partial():
    model = _model(freeze_encoders="none")
    from speech_transcript_embeddings_amd.train import FusedAdamW
    opt = FusedAdamW(model, lr=1e-3)
    assert opt.groups[0]["lr"] == opt.groups[1]["lr"] == 1e-3  # ref:1514-1519: one lr for everything
    opt.t = 1
    sd = opt.state_dict()
    assert len(sd["param_groups"]) == 1
    _ref_adamw(model, lr=1e-3, partial=False).load_state_dict(sd)


def test_checkpoint_round_trip(tmp_path):
    from speech_transcript_embeddings_amd.checkpoint import REF_KEYS, load_checkpoint, save_checkpoint
    model = _model("align")
    opt = _filled_opt(model)
    path = tmp_path / "best_model_loss.pt"
    d = save_checkpoint(path, model, opt, epoch=2, train_metrics={"loss": np.float64(0.7)},
                        val_metrics={"loss": 0.6, "similarity_gap": np.float32(0.1)}, temperature=0.1)
    assert tuple(d) == REF_KEYS
    raw = torch.load(path, weights_only=True)  # plain floats: loads with the strictest loader
    assert set(raw) == set(REF_KEYS) and raw["use_word_alignment"] is True
    assert raw["freeze_encoders"] == "partial" and raw["text_layers_to_unfreeze"] == model.text_layers_to_unfreeze
    fresh = _model("align")
    with torch.no_grad():
        for p in fresh.parameters():
            p.zero_()
    from speech_transcript_embeddings_amd.train import FusedAdamW
    opt2 = FusedAdamW(fresh)
    ck = load_checkpoint(path, fresh, opt2)
    assert ck["epoch"] == 2
    for (n, a), (_, b) in zip(model.state_dict().items(), fresh.state_dict().items()):
        assert torch.equal(a, b), n
    s1, s2 = opt.state_dict(), opt2.state_dict()  # every parameter's moments (the flat buffers' alignment
    assert opt2.t == 3 and s1["state"].keys() == s2["state"].keys()  # gaps are not state)
    for i, ps in s1["state"].items():
        assert torch.equal(ps["exp_avg"], s2["state"][i]["exp_avg"]) and torch.equal(ps["exp_avg_sq"],
                                                                                      s2["state"][i]["exp_avg_sq"])
    # strict load rejects a foreign tree
    sd = dict(ck["model_state_dict"])
    sd["not_a_parameter"] = torch.zeros(1)
    with pytest.raises(RuntimeError):
        fresh.load_state_dict(sd)


def test_reference_style_numpy_metrics_load_safely(tmp_path):
    """The reference's val_metrics hold numpy float64 (np.mean); torch.save pickles them."""
    from speech_transcript_embeddings_amd.checkpoint import load_checkpoint
    model = _model()
    path = tmp_path / "ref_style.pt"
    torch.save({"epoch": 1, "model_state_dict": model.state_dict(), "optimizer_state_dict": _ref_adamw(model).state_dict(),
                "train_metrics": {"loss": np.float64(1.0)}, "val_metrics": {"loss": np.mean([0.5, 0.7])},
                "temperature": 0.1}, path)
    with pytest.raises(Exception):
        torch.load(path, weights_only=True)
    ck = load_checkpoint(path, _model())
    assert float(ck["val_metrics"]["loss"]) == pytest.approx(0.6)
