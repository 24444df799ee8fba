"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Run only in the survey/build container (needs /root/reference and transformers):
    python tests/golden/make_golden.py

What it does (read-only use of /root/reference):
  * imports /root/reference/training/trainer_unfreeze.py with the four import
    shims SURVEY.md §8(c) lists (dotenv stub, HF_TOKEN dummy, get_device_name
    patch, no bytecode writes) and replaces its AutoModel with config-built
    encoders (no network: weights are deterministic, oracle/det_init.py);
  * fbank: runs transformers' SeamlessM4TFeatureExtractor (the arithmetic the
    reference calls at trainer_unfreeze.py:856-860) and the reference's
    custom_collate_fn on seeded synthetic clips -> fbank_golden.npz;
  * model: builds the reference EnhancedAudioTextModel at reduced dims (head_dim
    64 like the real encoders), eval mode, runs compute_pos_neg_embeddings ->
    s_pos/s_neg -> AlignmentAwareInfoNCE -> backward -> clip_grad_norm_ -> the
    reference's two-group AdamW + linear-warmup scheduler, and records outputs,
    per-tensor gradient norms/sums + sampled entries, and sampled post-step
    parameter values -> model_golden_<variant>.npz (+ .json config).
The fixtures are data only (inputs and expected outputs).
"""
from __future__ import annotations

import json
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
from oracle import det_init, fbank_ref  # noqa: E402

REF_TRAINING = "/root/reference/training"


def import_reference():
    sys.dont_write_bytecode = True
    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: None
    sys.modules["dotenv"] = dotenv
    os.environ.setdefault("HF_TOKEN", "dummy")
    torch.cuda.get_device_name = lambda *a, **k: "cpu"
    sys.path.insert(0, REF_TRAINING)
    import trainer_unfreeze as T  # noqa: E402
    return T


MINI = {
    "audio": dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                  feature_projection_input_dim=160, layerdrop=0.0, mask_time_prob=0.0,
                  left_max_position_embeddings=64, right_max_position_embeddings=8, conv_depthwise_kernel_size=31),
    "text": dict(vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=256, max_position_embeddings=514, type_vocab_size=1, layer_norm_eps=1e-5,
                 pad_token_id=1),
    "projection_dim": 128,
    "unfreeze": 1,
}


def make_automodel_shim(cfgs):
    from transformers import Wav2Vec2BertConfig, Wav2Vec2BertModel, XLMRobertaConfig, XLMRobertaModel

    class _Auto:
        @staticmethod
        def from_pretrained(name, *a, **k):
            if "w2v" in name:
                return Wav2Vec2BertModel(Wav2Vec2BertConfig(**cfgs["audio"]))
            return XLMRobertaModel(XLMRobertaConfig(**cfgs["text"]))
    return _Auto


def fbank_fixture(T):
    from transformers import SeamlessM4TFeatureExtractor
    fe = SeamlessM4TFeatureExtractor(feature_size=80, num_mel_bins=80, padding_value=1.0, sampling_rate=16000,
                                     stride=2)
    cases = [("2s", 1000, 32000), ("odd", 1001, 20000), ("short", 1002, 6000), ("1p3s", 1003, 20960)]
    out = {}
    waves = []
    for name, seed, n in cases:
        w = fbank_ref.synth_wave(seed, n)
        if name == "short":
            w[1000:3000] = 0.0  # an all-zero stretch: log-floor path
        if name == "1p3s":
            w = np.clip(w * 12.0, -3, 3).astype(np.float32)  # loud (> 1.0) clip
        r = fe(w, sampling_rate=16000, return_tensors="np")
        out[f"{name}_wave"] = w
        out[f"{name}_feats"] = r["input_features"][0].astype(np.float32)
        out[f"{name}_mask"] = r["attention_mask"][0].astype(np.int64)
        waves.append(w)
    # reference collate over extractor outputs (ids/masks dummy)
    items = []
    for name, _, _ in cases:
        items.append({
            "input_ids_pos": torch.zeros(4, dtype=torch.long), "attention_mask_pos": torch.ones(4, dtype=torch.long),
            "input_ids_neg": torch.zeros(4, dtype=torch.long), "attention_mask_neg": torch.ones(4, dtype=torch.long),
            "input_values": torch.from_numpy(out[f"{name}_feats"]),
            "attention_mask_audio": torch.from_numpy(out[f"{name}_mask"])})
    batch = T.custom_collate_fn(items)
    out["batch_feats"] = batch["input_values"].numpy()
    out["batch_mask"] = batch["attention_mask_audio"].numpy()
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(HERE / "fbank_golden.npz", **out)
    print("fbank_golden.npz", {k: v.shape for k, v in out.items()})


def fbank_long_fixture(T):
    """Config-size clips (tests/golden/fbank_cases.py): the reference extractor's features/masks
    and the reference collate over all of them -> fbank_golden_long.npz (waveforms rebuilt from
    seeds by the tests, not stored)."""
    from transformers import SeamlessM4TFeatureExtractor
    sys.path.insert(0, str(HERE))
    from fbank_cases import LONG_CASES, long_case_wave
    fe = SeamlessM4TFeatureExtractor(feature_size=80, num_mel_bins=80, padding_value=1.0, sampling_rate=16000,
                                     stride=2)
    out, items = {}, []
    for name, _, _ in LONG_CASES:
        r = fe(long_case_wave(name), sampling_rate=16000, return_tensors="np")
        out[f"{name}_feats"] = r["input_features"][0].astype(np.float32)
        out[f"{name}_mask"] = r["attention_mask"][0].astype(np.int64)
        items.append({
            "input_ids_pos": torch.zeros(4, dtype=torch.long), "attention_mask_pos": torch.ones(4, dtype=torch.long),
            "input_ids_neg": torch.zeros(4, dtype=torch.long), "attention_mask_neg": torch.ones(4, dtype=torch.long),
            "input_values": torch.from_numpy(out[f"{name}_feats"]),
            "attention_mask_audio": torch.from_numpy(out[f"{name}_mask"])})
    batch = T.custom_collate_fn(items)
    out["batch_mask"] = batch["attention_mask_audio"].numpy()
    out["cases"] = np.array([c[0] for c in LONG_CASES])
    np.savez_compressed(HERE / "fbank_golden_long.npz", **out)
    print("fbank_golden_long.npz", {k: v.shape for k, v in out.items()})


def synth_batch(T, B=2, L=12, vocab=1000, masked=False):
    from transformers import SeamlessM4TFeatureExtractor
    fe = SeamlessM4TFeatureExtractor(feature_size=80, num_mel_bins=80, padding_value=1.0, sampling_rate=16000,
                                     stride=2)
    lens = [16000, 12800, 9600][:B]
    rng = np.random.default_rng(77)
    items = []
    for i in range(B):
        w = fbank_ref.synth_wave(500 + i, lens[i])
        r = fe(w, sampling_rate=16000, return_tensors="pt")
        n_tok = L - 3 * i
        ids = rng.integers(5, vocab, size=L)
        ids[0], ids[n_tok - 1] = 0, 2
        ids[n_tok:] = 1
        mask = np.zeros(L, np.int64); mask[:n_tok] = 1
        neg = ids.copy()
        sel = rng.random(L) < 0.3
        sel[0] = False; sel[n_tok - 1:] = False
        neg[sel] = rng.integers(5, vocab, size=int(sel.sum()))
        items.append({
            "input_ids_pos": torch.from_numpy(ids), "attention_mask_pos": torch.from_numpy(mask),
            "input_ids_neg": torch.from_numpy(neg), "attention_mask_neg": torch.from_numpy(mask.copy()),
            "input_values": r["input_features"][0], "attention_mask_audio": r["attention_mask"][0]})
    batch = T.custom_collate_fn(items)
    if masked:   # edge cases of the masks: sample 1's transcripts and sample 2's audio fully masked
        batch["attention_mask_pos"][1] = 0
        batch["attention_mask_neg"][1] = 0
        batch["attention_mask_audio"][2] = 0
    return batch


def model_fixture(T, use_align: bool, attentive: bool = True, masked: bool = False):
    T.AutoModel = make_automodel_shim(MINI)
    torch.manual_seed(0)
    model = T.EnhancedAudioTextModel(
        text_model_name="xlmr-mini", audio_model_name="w2v-bert-mini",
        projection_dim=MINI["projection_dim"], text_embedding_dim=MINI["text"]["hidden_size"],
        audio_embedding_dim=MINI["audio"]["hidden_size"], dropout=0.1, use_cross_modal=True,
        use_attentive_pooling=attentive, use_word_alignment=use_align, freeze_encoders="partial",
        text_layers_to_unfreeze=MINI["unfreeze"], audio_layers_to_unfreeze=MINI["unfreeze"])
    sd = model.state_dict()
    vals = det_init.state_dict_values([(n, t.shape) for n, t in sd.items() if t.is_floating_point()])
    model.load_state_dict({n: torch.from_numpy(v) for n, v in vals.items()}, strict=False)
    model.eval()
    batch = synth_batch(T, B=3, masked=True) if masked else synth_batch(T)
    tpn, tnn, an = T.EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
    s_pos = (an * tpn).sum(1)
    s_neg = (an * tnn).sum(1)
    align = getattr(model, "last_alignment_scores", None)
    loss_fn = T.AlignmentAwareInfoNCE(temperature=0.1, alignment_weight=0.5)
    loss = loss_fn(s_pos, s_neg, alignment_scores=align)
    (loss / 1.0).backward()

    out = {k: v.numpy() for k, v in batch.items()}
    out.update(txt_pos=tpn.detach().numpy(), txt_neg=tnn.detach().numpy(), aud=an.detach().numpy(),
               s_pos=s_pos.detach().numpy(), s_neg=s_neg.detach().numpy(), loss=np.float32(loss.item()))
    if align is not None:
        out["align"] = align.detach().numpy()
    names = [n for n, p in model.named_parameters()]
    trainable = [n for n, p in model.named_parameters() if p.requires_grad]
    with_grad = [n for n, p in model.named_parameters() if p.grad is not None]
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().reshape(-1).numpy()
        idx = det_init.sample_indices(n, g.size)
        out[f"gnorm::{n}"] = np.float64(np.linalg.norm(g.astype(np.float64)))
        out[f"gsum::{n}"] = np.float64(g.astype(np.float64).sum())
        out[f"gsamp::{n}"] = g[idx]
    # ---- reference optimizer tail: clip + two-group AdamW + linear warmup (ref:1487-1541, 1108-1113)
    lr = 2.1e-3
    enc, head = [], []
    for n, p in model.named_parameters():
        if p.requires_grad:
            (enc if ("text_encoder" in n or "audio_encoder" in n) else head).append(p)
    opt = torch.optim.AdamW([{"params": enc, "lr": lr / 50, "weight_decay": 0.01},
                             {"params": head, "lr": lr, "weight_decay": 0.01}])
    from transformers import get_linear_schedule_with_warmup
    sched = get_linear_schedule_with_warmup(opt, num_warmup_steps=2, num_training_steps=10)
    sched.step()  # lr(step 0) == 0 in the reference; take the step at scheduler step 1
    total_norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
    out["clip_total_norm"] = np.float64(total_norm.item())
    out["lr_enc"] = np.float64(opt.param_groups[0]["lr"])
    out["lr_head"] = np.float64(opt.param_groups[1]["lr"])
    opt.step()
    for n, p in model.named_parameters():
        if p.grad is None:
            continue
        idx = det_init.sample_indices(n, p.numel())
        out[f"pnew::{n}"] = p.detach().reshape(-1).numpy()[idx]
    cfg = {"mini": MINI, "use_word_alignment": use_align, "use_attentive_pooling": attentive, "names": names, "trainable": trainable,
           "with_grad": with_grad, "lr": lr, "warmup": 2, "total_steps": 10, "sched_step": 1,
           "param_count": sum(p.numel() for p in model.parameters()),
           "trainable_count": sum(p.numel() for p in model.parameters() if p.requires_grad)}
    tag = "masked" if masked else ("align" if use_align else "noalign") if attentive else "nopool"
    np.savez_compressed(HERE / f"model_golden_{tag}.npz", **out)
    (HERE / f"model_golden_{tag}.json").write_text(json.dumps(cfg, indent=1))
    print(f"model_golden_{tag}.npz loss={loss.item():.6f} trainable={cfg['trainable_count']}")


def param_count_fixture(T):
    """Full-size module trees (random init, meta-free CPU) -> exact parameter counts the logs report."""
    from transformers import Wav2Vec2BertConfig, XLMRobertaConfig
    full = {"audio": Wav2Vec2BertConfig().to_dict(),
            "text": dict(vocab_size=250002, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                         intermediate_size=3072, max_position_embeddings=514, type_vocab_size=1,
                         layer_norm_eps=1e-5, pad_token_id=1)}
    full["audio"] = {k: v for k, v in full["audio"].items() if k in Wav2Vec2BertConfig().to_dict()}
    res = {}
    for align, k in [(False, 3), (True, 3), (True, 5)]:
        T.AutoModel = make_automodel_shim(full)
        m = T.EnhancedAudioTextModel(text_model_name="mpnet", audio_model_name="facebook/w2v-bert-2.0",
                                     use_word_alignment=align, text_layers_to_unfreeze=k,
                                     audio_layers_to_unfreeze=k)
        res[f"align={align},k={k}"] = {
            "total": sum(p.numel() for p in m.parameters()),
            "trainable": sum(p.numel() for p in m.parameters() if p.requires_grad),
            "shapes": {n: list(p.shape) for n, p in m.named_parameters()},
            "trainable_names": [n for n, p in m.named_parameters() if p.requires_grad]}
        del m
    (HERE / "param_counts.json").write_text(json.dumps(res))
    print({k: (v["total"], v["trainable"]) for k, v in res.items()})


if __name__ == "__main__":
    T = import_reference()
    if "--fbank-long" in sys.argv:  # only the config-size fbank fixture
        fbank_long_fixture(T)
        sys.exit(0)
    if "--masked" in sys.argv:      # only the all-masked-sample model fixture
        model_fixture(T, use_align=False, masked=True)
        sys.exit(0)
    fbank_fixture(T)
    fbank_long_fixture(T)
    model_fixture(T, use_align=False)
    model_fixture(T, use_align=True)
    model_fixture(T, use_align=False, attentive=False)  # CLS text / masked-mean audio (ref:578-580,621-636)
    model_fixture(T, use_align=False, masked=True)      # fully masked transcripts / audio of one sample
    if "--counts" in sys.argv:
        param_count_fixture(T)
