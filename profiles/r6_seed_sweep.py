"""(Round 6 copy of profiles/r5_seed_sweep.py, with per-tensor excess statistics over ALL audio tensors
and over all distance tables.)  HIP vs same-instance bf16 floor over several draws (weights, clips, cotangents) of the
full-size parity configs: how much of a single instance's HIP-minus-floor is draw noise, and
which excess is systematic.  Test tooling: reuses tests/test_fullsize_gpu.py's instance builder
and floor emulation; run on the GPU box:  python profiles/r5_seed_sweep.py [--configs c1,c2,c5] [--seeds 6]"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import test_fullsize_gpu as T  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="c1,c2,c4,c5")
ap.add_argument("--seeds", type=int, default=6)
args = ap.parse_args()
for cname in args.configs.split(","):
    for s in range(args.seeds):
        r = T._hip_vs_oracle(cname, model_seed=100 + s, data_seed=200 + s, cot_seed=300 + s)
        floor, _ = T._floor_errs(r["sd"], r["bc"]["input_values"], r["cfg"].audio, r["trainable"], r["cap"])
        skip = ("linear_k.bias", "attention.2.bias")
        aud = [(e, n) for e, n in r["errs"] if n.startswith(("audio_encoder.", "audio_pooling.")) and not n.endswith(skip)]
        rest = [(e, n) for e, n in r["errs"] if not n.startswith(("audio_encoder.", "audio_pooling."))]
        fl = sorted(((e, n) for n, e in floor.items() if not n.endswith(skip)), reverse=True)
        diffs = sorted(((e - floor[n], n) for e, n in aud if n in floor), reverse=True)
        dist = [(round(e, 5), round(floor.get(n, float("nan")), 5), n.replace("audio_encoder.encoder.", ""))
                for e, n in aud if "distance_embedding" in n][:4]
        print(json.dumps({"config": cname, "seed": s, "hip_worst_audio": [round(aud[0][0], 5), aud[0][1]],
                          "floor_worst": [round(fl[0][0], 5), fl[0][1]],
                          "hip_minus_floor_worst_audio": round(aud[0][0] - fl[0][0], 5),
                          "largest_per_tensor_excess": [(round(d, 5), n.replace("audio_encoder.encoder.", ""))
                                                        for d, n in diffs[:3]],
                          "distance_tables": dist,
                          "per_tensor_excess_all_audio": {"mean": round(sum(d for d, _ in diffs) / len(diffs), 5),
                                                          "max": round(diffs[0][0], 5), "min": round(diffs[-1][0], 5),
                                                          "n": len(diffs)},
                          "per_tensor_excess_distance_tables": (lambda dd: {"mean": round(sum(dd) / len(dd), 5),
                                                                            "max": round(max(dd), 5),
                                                                            "min": round(min(dd), 5), "n": len(dd)})(
                              [d for d, n in diffs if "distance_embedding" in n]),
                          "non_audio_worst": [round(rest[0][0], 5), rest[0][1]] if rest else None}), flush=True)
