"""Collect the round-6 parity record (profiles/r6_parity.txt) from `pytest -m gpu -v -s` logs.

Keeps every line a parity test prints about its own errors — the GEMM instantiation table
("[r6 gemm spec] ..."), the full-size per-draw floors and excesses ("[c2-d1] ..."), the plan
equivalence figures, the alignment-head floor — and each log's pass/fail summary line.

    python profiles/r6_parity.py OUT.txt LOG [LOG ...]
"""
import re
import sys

HEADER = """Round 6 parity record (tests' own printed figures, per GPU log below).
Per-tensor gradient errors are relative L2 norms vs the fp32/fp64 reference on the same bf16-exact
operands unless stated.  'floor' = the same-instance bf16 floor: the HIP path's rounding points
emulated on the CPU on the test's own weights, inputs and cotangents (tests/precision_probe.py,
precision_probe_align.py; DESIGN §4); 'excess' = HIP error - floor, per tensor, in points (1e-2).
GEMM spec lines: each compile-time epilogue instantiation of the bench plan (>= 240 tiles, the
kernel name asserted) vs fp64 on the same bf16 operands; C / C2 / C3 = each output's relative
error (bf16 outputs carry their own rounding, ~1.7e-3).
"""

TAG = re.compile(r"(\[(r6 |c\d|plan|head|align|fp8|mx|gemm|equiv)[^\]]*\].*)$")


def main():
    out, logs = sys.argv[1], sys.argv[2:]
    lines = [HEADER]
    for path in logs:
        lines.append(f"\n=== {path}")
        cur = None
        for raw in open(path, errors="replace"):
            raw = raw.rstrip("\n")
            m = re.match(r"^(tests/\S+::\S+)", raw)
            if m:
                cur = m.group(1)
            t = TAG.search(raw.split(" PASSED")[0].split(" FAILED")[0])
            if t and not raw.startswith("[r6] ") and not t.group(1).startswith("[c10d]") \
                    and t.group(1).rstrip("] [").strip() not in ("[align", "[align]"):
                lines.append(t.group(1))
            if re.search(r"=+ .*(passed|failed).* =+", raw):
                lines.append(raw.strip("= "))
            if cur and raw.rstrip().endswith("FAILED"):
                lines.append(f"FAILED {cur}")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
