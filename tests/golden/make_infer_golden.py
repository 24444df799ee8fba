"""Golden vectors for the inference model variant (reference model.py:131-329,
EnhancedAudioTextModel.forward used by inference.py:48-120): the REAL reference model.py at mini
dimensions (RoBERTa / w2v-bert encoders built from configs through an AutoModel shim, weights
from oracle/det_init.py), eval mode, forward(batch) -> (text_embeddings, audio_embeddings).

Run only in the build container (needs /root/reference and transformers):
    python tests/golden/make_infer_golden.py
Writes infer_golden.npz (inputs + outputs) and infer_golden.json (config + parameter names).
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

TEXT = dict(vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
            max_position_embeddings=514, type_vocab_size=1, layer_norm_eps=1e-5, pad_token_id=1)


def main():
    T = import_reference()  # only for custom_collate_fn / the shared batch maker
    import transformers
    from transformers import RobertaConfig, RobertaModel, Wav2Vec2BertConfig, Wav2Vec2BertModel

    def from_pretrained(name, *a, **k):  # config-built encoders, no download
        if "w2v" in name:
            return Wav2Vec2BertModel(Wav2Vec2BertConfig(**MINI["audio"]))
        return RobertaModel(RobertaConfig(**TEXT))

    transformers.AutoModel.from_pretrained = staticmethod(from_pretrained)
    sys.path.insert(0, "/root/reference")
    import model as RM  # reference model.py (inference variant)
    torch.manual_seed(0)
    m = RM.EnhancedAudioTextModel(text_model_name="roberta-mini", audio_model_name="w2v-bert-mini",
                                  projection_dim=128, text_embedding_dim=128, audio_embedding_dim=128, dropout=0.1,
                                  use_cross_modal=True, use_attentive_pooling=True, freeze_encoders=True)
    sd = m.state_dict()
    vals = det_init.state_dict_values([(n, t.shape) for n, t in sd.items() if t.is_floating_point()])
    m.load_state_dict({n: torch.from_numpy(v) for n, v in vals.items()}, strict=False)
    m.eval()
    b = synth_batch(T)
    batch = {"input_ids": b["input_ids_pos"], "attention_mask": b["attention_mask_pos"],
             "input_features": b["input_values"], "attention_mask_audio": b["attention_mask_audio"]}
    with torch.no_grad():
        te, ae = m(batch)
        tp, th = m.encode_text(batch["input_ids"], batch["attention_mask"])
        ap, ah = m.encode_audio(batch["input_features"], batch["attention_mask_audio"])
    out = {k: v.numpy() for k, v in batch.items()}
    out.update(text_emb=te.numpy(), audio_emb=ae.numpy(), text_proj=tp.numpy(), audio_proj=ap.numpy(),
               text_hidden=th.numpy(), audio_hidden=ah.numpy())
    np.savez_compressed(HERE / "infer_golden.npz", **out)
    meta = {"source": "model.py:131-329", "text": TEXT, "audio": MINI["audio"], "projection_dim": 128,
            "names": list(sd.keys()), "shapes": {n: list(t.shape) for n, t in sd.items()},
            "trainable": [n for n, p in m.named_parameters() if p.requires_grad]}
    (HERE / "infer_golden.json").write_text(json.dumps(meta, indent=0))
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
