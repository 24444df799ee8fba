"""Which of the attention's own approximations puts the HIP path above the same-instance bf16
floor (tests/test_fullsize_gpu.py) at c5 / c1?  Runs the full-size comparison once, then the floor
emulation with extra rounding points (precision_probe.Probe olo / plo) on the same instance, and
prints, for the HIP path's worst audio tensors, HIP error / emulated error per variant.

    python profiles/r5_floor_diag.py c5 [c1 ...]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import test_fullsize_gpu as TF  # noqa: E402

VARIANTS = {"floor": None, "olo_bf16": dict(olo="bf16"), "olo_fp16s": dict(olo="fp16s"), "plo": dict(plo=True),
            "plo+olo_bf16": dict(plo=True, olo="bf16")}

for cname in sys.argv[1:] or ["c5"]:
    r = TF._hip_vs_oracle(cname)
    aud = [(e, n) for e, n in r["errs"] if n.startswith(("audio_encoder.", "audio_pooling."))][:10]
    res = {}
    for vn, kw in VARIANTS.items():
        res[vn], _ = TF._floor_errs(r["sd"], r["bc"]["input_values"], r["cfg"].audio, r["trainable"], r["cap"], kw)
        worst = sorted(((e, n) for n, e in res[vn].items() if not n.endswith(("linear_k.bias", "attention.2.bias"))),
                       reverse=True)[:3]
        print(f"[{cname}] {vn}: emulated worst " + ", ".join(f"{n.replace('audio_encoder.encoder.', '')} {e:.4f}"
                                                         for e, n in worst), flush=True)
    print(f"[{cname}] tensor: HIP | " + " | ".join(VARIANTS))
    for e, n in aud:
        print(f"  {n.replace('audio_encoder.encoder.', '')}: {e:.4f} | "
              + " | ".join(f"{res[v].get(n, float('nan')):.4f}" for v in VARIANTS), flush=True)
