"""Reduce two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs of
`bench.py --steps 1 --warmup 1`) to per-launch HBM traffic per kernel.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of
wide coalesced reads -> x2; WRITE_SIZE is exact for 16-B stores.  Both counters are in KiB.
Only the dispatches of the last step are used (from the last fbank_tables_kernel launch,
the first kernel of every step, to the end).

    python profiles/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/r1_hbm_traffic.json
"""
import csv
import json
import re
import sys
from collections import defaultdict


def load(d, counter):
    rows = [r for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    start = max(i for i, r in enumerate(rows) if "fbank_tables_kernel" in r["Kernel_Name"])
    return rows[start:]


def short(name):
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:80]


def main(fd, wd):
    acc = defaultdict(lambda: [0, 0.0, 0.0])
    for r in load(fd, "FETCH_SIZE"):
        a = acc[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += 2.0 * float(r["Counter_Value"]) * 1024
    for r in load(wd, "WRITE_SIZE"):
        acc[short(r["Kernel_Name"])][2] += float(r["Counter_Value"]) * 1024
    out = {k: {"launches": n, "fetch_bytes_per_launch": round(f / n), "write_bytes_per_launch": round(w / n),
               "hbm_bytes_per_launch": round((f + w) / n)} for k, (n, f, w) in acc.items() if n}
    print(json.dumps(dict(sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"])),
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
