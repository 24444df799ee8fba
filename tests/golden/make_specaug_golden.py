"""Golden vectors for SpecAugment in training mode (w2v-bert time masking,
tf:models/wav2vec2_bert/modeling_wav2vec2_bert.py:800-988, on by default when the reference
trains): the REAL reference trainer model at mini dims, train mode with every dropout at 0 so
that the only randomness is SpecAugment's numpy draws, np.random.seed(SEED) right before
compute_pos_neg_embeddings -> loss -> backward.  Also records the span mask transformers'
own _compute_mask_indices draws from the same seed.

Run only in the build container (needs /root/reference and transformers):
    python tests/golden/make_specaug_golden.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.dont_write_bytecode = True
from oracle import det_init  # noqa: E402
from make_golden import MINI, import_reference, synth_batch  # noqa: E402

SEED = 1234
AUDIO = dict(MINI["audio"], mask_time_prob=0.3, mask_time_length=4, mask_time_min_masks=2, hidden_dropout=0.0,
             attention_dropout=0.0, activation_dropout=0.0, feat_proj_dropout=0.0, conformer_conv_dropout=0.0,
             layerdrop=0.0)
TEXT = dict(MINI["text"], hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


def main():
    T = import_reference()
    from transformers import Wav2Vec2BertConfig, Wav2Vec2BertModel, XLMRobertaConfig, XLMRobertaModel
    from transformers.models.wav2vec2_bert import modeling_wav2vec2_bert as W

    class _Auto:
        @staticmethod
        def from_pretrained(name, *a, **k):
            if "w2v" in name:
                return Wav2Vec2BertModel(Wav2Vec2BertConfig(**AUDIO))
            return XLMRobertaModel(XLMRobertaConfig(**TEXT))

    T.AutoModel = _Auto
    torch.manual_seed(0)
    model = T.EnhancedAudioTextModel(
        text_model_name="xlmr-mini", audio_model_name="w2v-bert-mini", projection_dim=MINI["projection_dim"],
        text_embedding_dim=MINI["text"]["hidden_size"], audio_embedding_dim=MINI["audio"]["hidden_size"], dropout=0.0,
        use_cross_modal=True, use_attentive_pooling=True, use_word_alignment=False, freeze_encoders="partial",
        text_layers_to_unfreeze=MINI["unfreeze"], audio_layers_to_unfreeze=MINI["unfreeze"])
    sd = model.state_dict()
    vals = det_init.state_dict_values([(n, t.shape) for n, t in sd.items() if t.is_floating_point()])
    model.load_state_dict({n: torch.from_numpy(v) for n, v in vals.items()}, strict=False)
    model.train()
    batch = synth_batch(T)
    np.random.seed(SEED)
    tpn, tnn, an = T.EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
    s_pos, s_neg = (an * tpn).sum(1), (an * tnn).sum(1)
    loss = T.AlignmentAwareInfoNCE(temperature=0.1, alignment_weight=0.5)(s_pos, s_neg)
    loss.backward()
    am = batch["attention_mask_audio"]
    np.random.seed(SEED)
    spec = W._compute_mask_indices(tuple(am.shape), mask_prob=AUDIO["mask_time_prob"],
                                   mask_length=AUDIO["mask_time_length"], attention_mask=am,
                                   min_masks=AUDIO["mask_time_min_masks"])
    out = {k: v.numpy() for k, v in batch.items()}
    out.update(txt_pos=tpn.detach().numpy(), txt_neg=tnn.detach().numpy(), aud=an.detach().numpy(),
               loss=np.float32(loss.item()), spec_mask=spec)
    grads = {}
    for n, p in model.named_parameters():
        if p.grad is not None:
            g = p.grad.detach().reshape(-1).numpy()
            grads[n] = g
            out[f"gnorm::{n}"] = np.float64(np.linalg.norm(g.astype(np.float64)))
    out["g::audio_encoder.masked_spec_embed"] = grads["audio_encoder.masked_spec_embed"]
    np.savez_compressed(HERE / "specaug_golden.npz", **out)
    meta = {"seed": SEED, "audio": AUDIO, "text": TEXT, "mini": MINI, "use_word_alignment": False,
            "with_grad": sorted(grads), "names": list(sd.keys())}
    (HERE / "specaug_golden.json").write_text(json.dumps(meta, indent=0))
    print("spec rows masked:", int(spec.sum()), "of", spec.size, "; loss", loss.item())


if __name__ == "__main__":
    main()
