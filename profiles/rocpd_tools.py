"""Reduce rocprofv3 rocpd databases (ROCm 7.2 default output, `run_results.db`) to the
committed summaries under profiles/.

  kernel stats  (same columns as rocprofv3 --stats kernel_stats.csv):
    python profiles/rocpd_tools.py stats gpurun_out/prof/run_results.db > profiles/rNN_bench_kernel_stats.csv
  per-kernel means of SQ counters from --pmc passes (e.g. of profiles/attn_probe.py):
    python profiles/rocpd_tools.py pmc gpurun_out/p1/run_results.db gpurun_out/p2/run_results.db
  per-launch HBM traffic from separate FETCH_SIZE / WRITE_SIZE passes of bench.py:
    python profiles/rocpd_tools.py traffic gpurun_out/pmc_fetch/run_results.db gpurun_out/pmc_write/run_results.db \
        > profiles/rNN_hbm_traffic.json

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of wide
coalesced reads -> x2; WRITE_SIZE is exact for 16-B stores; both counters are in KiB.  For traffic
only the dispatches of the last step are used (from the last fbank_logmel_kernel launch, the
first kernel of every step, to the end).
"""
import csv
import json
import math
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:80]


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels").fetchall()
    acc = defaultdict(list)
    for n, d in rows:
        acc[n].append(float(d))
    total = sum(sum(v) for v in acc.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        s, k = sum(v), len(v)
        mu = s / k
        sd = math.sqrt(sum((x - mu) ** 2 for x in v) / k)
        w.writerow([n, k, int(s), round(mu, 3), round(100 * s / total, 2), int(min(v)), int(max(v)), round(sd, 3)])


def _grid_col(c):
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)").fetchall()]
    for n in ("grid_size", "grid_size_x", "grid_x"):
        if n in cols:
            return n
    return None


def counter(db, name, with_grid=False):
    """[(kernel, value)] (or [(kernel, grid, value)]) per dispatch of the last step."""
    c = sqlite3.connect(db)
    gc = _grid_col(c) if with_grid else None
    sel = f"dispatch_id, kernel_name, {gc if gc else '0'}, value"
    rows = c.execute(f"select {sel} from counters_collection where counter_name = ?", (name,)).fetchall()
    agg = defaultdict(lambda: [None, 0, 0.0])
    for d, k, gr, v in rows:
        a = agg[d]
        a[0], a[1] = k, gr
        a[2] += float(v)
    out = sorted(agg.items())
    start = max(i for i, (_, (k, _, _)) in enumerate(out) if "fbank_logmel_kernel" in k)
    if with_grid:
        return [(k, gr, v) for _, (k, gr, v) in out[start:]]
    return [(k, v) for _, (k, _, v) in out[start:]]


def traffic(fdb, wdb):
    acc = defaultdict(lambda: [0, 0.0, 0.0])
    for k, v in counter(fdb, "FETCH_SIZE"):
        a = acc[short(k)]
        a[0] += 1
        a[1] += 2.0 * v * 1024
    for k, v in counter(wdb, "WRITE_SIZE"):
        acc[short(k)][2] += v * 1024
    out = {k: {"launches": n, "fetch_bytes_per_launch": round(f / n), "write_bytes_per_launch": round(w / n),
               "hbm_bytes_per_launch": round((f + w) / n)} for k, (n, f, w) in acc.items() if n}
    res = dict(sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]))
    # the same per launch population: kernel name + grid size (work-items), so that one kernel's
    # launches at different shapes (audio vs text rows, main vs side stream) can be compared with
    # bench.py's per-shape algorithmic bytes
    byg = defaultdict(lambda: [0, 0.0, 0.0])
    for k, gr, v in counter(fdb, "FETCH_SIZE", True):
        a = byg[f"{short(k)}@{gr}"]
        a[0] += 1
        a[1] += 2.0 * v * 1024
    for k, gr, v in counter(wdb, "WRITE_SIZE", True):
        byg[f"{short(k)}@{gr}"][2] += v * 1024
    res["by_grid"] = {k: {"launches": n, "fetch_bytes_per_launch": round(f / n), "write_bytes_per_launch": round(w / n),
                          "hbm_bytes_per_launch": round((f + w) / n)}
                      for k, (n, f, w) in sorted(byg.items(), key=lambda kv: -(kv[1][1] + kv[1][2])) if n}
    print(json.dumps(res, indent=1))


def pmc(*dbs):
    """Per-kernel mean of every collected counter (one row per kernel, one column per counter)
    over all dispatches of one or more --pmc passes."""
    acc = defaultdict(lambda: defaultdict(list))
    for db in dbs:
        c = sqlite3.connect(db)
        rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
        per = defaultdict(float)
        names = {}
        for d, k, cn, v in rows:
            per[(d, cn)] += float(v)
            names[d] = k
        for (d, cn), v in per.items():
            acc[short(names[d])][cn].append(v)
    out = {k: {cn: round(sum(v) / len(v), 1) for cn, v in sorted(cs.items())} for k, cs in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2])
    elif sys.argv[1] == "pmc":
        pmc(*sys.argv[2:])
    else:
        traffic(sys.argv[2], sys.argv[3])
