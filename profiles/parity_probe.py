"""Parity table of the loss-derived gradients (GPU, test infrastructure): the drop-in autograd path
(compute_pos_neg_embeddings -> (a*t).sum(1) -> AlignmentAwareInfoNCE -> backward, ref
trainer_unfreeze.py:1068-1094) on the golden mini batches against the CPU fp32 oracle (pinned to
the reference by tests/golden), per parameter tensor:
  elem  = ||g_hip - g_ref|| / ||g_ref||           (elementwise relative L2)
  norm  = | ||g_hip|| - ||g_ref|| | / ||g_ref||   (north_star's per-tensor bound: 1e-2 bf16)
  sign  = fraction of entries with the same sign  (AdamW's first step moves each by ±lr·sign)
Usage (on the GPU box): python profiles/parity_probe.py [--json out.json]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from test_model_gpu import batch_of, load, mini_model
    from oracle import det_init, ref_model as R
    from speech_transcript_embeddings_amd.model import AlignmentAwareInfoNCE, EnhancedAudioTextModel
    report = {}
    for tag in ("noalign", "align", "nopool", "masked"):
        meta, z = load(tag)
        model = mini_model(meta)
        model.eval()
        batch = batch_of(z)
        tpn, tnn, an = EnhancedAudioTextModel.compute_pos_neg_embeddings(model, batch)
        loss = AlignmentAwareInfoNCE(0.1, 0.5)((an * tpn).sum(1), (an * tnn).sum(1),
                                               alignment_scores=model.last_alignment_scores)
        loss.backward()
        torch.cuda.synchronize()
        cfg = R.mini_cfg(meta)
        vals = det_init.state_dict_values(R.param_shapes(cfg, spec_augment=False))
        p = {n: torch.from_numpy(v).requires_grad_(n in set(meta["trainable"])) for n, v in vals.items()}
        bc = {k: torch.from_numpy(z[k]) for k in ["input_ids_pos", "attention_mask_pos", "input_ids_neg",
                                                   "attention_mask_neg", "input_values", "attention_mask_audio"]}
        lo, *_ = R.step_loss(p, bc, cfg)
        lo.backward()
        params = dict(model.named_parameters())
        rows = []
        agree = total = sagree = stotal = 0
        for n in meta["with_grad"]:
            gr = p[n].grad.double().reshape(-1)
            if gr.norm() < 1e-6:
                continue   # analytically zero (softmax-shift-invariant key biases)
            gh = params[n].grad.detach().double().cpu().reshape(-1)
            e = ((gh - gr).norm() / gr.norm()).item()
            ne = abs(gh.norm().item() - gr.norm().item()) / gr.norm().item()
            sg = (torch.sign(gh) == torch.sign(gr)).double()
            idx = torch.from_numpy(det_init.sample_indices(n, gr.numel()))
            agree += int(sg.sum())
            total += sg.numel()
            sagree += int(sg[idx].sum())
            stotal += idx.numel()
            rows.append((n, e, ne, sg.mean().item()))
        # the fused TrainStep (bench path) on the same batch: accumulation window of 2, so its
        # gradient (x 1/2) is left in the flat buffer without an optimizer step
        from speech_transcript_embeddings_amd.train import TrainStep
        m2 = mini_model(meta, spec_augment=False)
        m2.dropout = 0.0
        m2.audio_cfg.conformer_conv_dropout = 0.0
        m2.audio_cfg.layerdrop = 0.0
        m2.text_cfg.hidden_dropout_prob = 0.0
        m2.text_cfg.attention_probs_dropout_prob = 0.0
        ts = TrainStep(m2, accumulation_steps=2)
        ts.step_batch(batch_of(z))
        torch.cuda.synchronize()
        fagree = ftotal = 0
        fworst = 0.0
        for n in meta["with_grad"]:
            gr = p[n].grad.double().reshape(-1)
            if gr.norm() < 1e-6:
                continue
            gf = m2.store.g(n).double().cpu().reshape(-1) * 2.0
            fworst = max(fworst, ((gf - gr).norm() / gr.norm()).item())
            sg = (torch.sign(gf) == torch.sign(gr)).double()
            fagree += int(sg.sum())
            ftotal += sg.numel()
        rows.sort(key=lambda r: -r[1])
        els = sorted(r[1] for r in rows)
        nes = sorted(r[2] for r in rows)
        summ = {"loss_hip": loss.item(), "loss_ref": lo.item(), "tensors": len(rows),
                "elem_median": els[len(els) // 2], "elem_worst": els[-1], "norm_median": nes[len(nes) // 2],
                "norm_worst": nes[-1], "sign_all": agree / total, "sign_sampled": sagree / stotal,
                "trainstep_elem_worst": fworst, "trainstep_sign_all": fagree / ftotal}
        print(f"== {tag}: {json.dumps(summ)}")
        print(f"{'tensor':70s} {'elem':>8s} {'norm':>8s} {'sign':>7s}")
        for n, e, ne, s in rows[:25]:
            print(f"{n:70s} {e:8.4f} {ne:8.4f} {s:7.4f}")
        report[tag] = {"summary": summ, "rows": rows}
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
