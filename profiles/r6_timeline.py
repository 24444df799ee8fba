"""Where the c2 step's wall time goes between kernels (profiling tooling, CPU side).

Reads a rocprofv3 --kernel-trace CSV (profiles/profile_bench.sh: gpurun_out/prof_TAG/trace/.../
run_kernel_trace.csv) of `bench.py --steps S --warmup W --trace-steps 2` and reports, over the last
`--window-ms` of the run (the timed steps and the two traced ones; warm-up and set-up excluded):
  * per queue (stream): busy time (union of its kernel intervals) and kernel count;
  * the GPU-busy time (union over all queues) and the idle remainder;
  * the largest idle gaps on the busiest (main) queue, with the kernels on either side.

    python profiles/r6_timeline.py TRACE.csv [--window-ms 1000] [--steps 7]
"""
import argparse
import csv
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=1000.0)
    ap.add_argument("--steps", type=int, default=7, help="steps inside the window (for per-step figures)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    key_q = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key_q], r["Kernel_Name"]) for r in rows]
    end = max(k[1] for k in ks)
    t0 = end - int(a.window_ms * 1e6)
    ks = [k for k in ks if k[0] >= t0]
    span = (max(k[1] for k in ks) - min(k[0] for k in ks)) / 1e6
    byq = defaultdict(list)
    for s, e, q, n in ks:
        byq[q].append((s, e, n))
    print(f"window {span:.1f} ms, {len(ks)} kernels, {a.steps} steps -> {span / a.steps:.2f} ms/step")
    main_q = max(byq, key=lambda q: sum(e - s for s, e, _ in byq[q]))
    for q, lst in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        busy = sum(b - a_ for a_, b in union([(s, e) for s, e, _ in lst])) / 1e6
        print(f"queue {q}{' (main)' if q == main_q else ''}: {len(lst)} kernels, busy {busy:.1f} ms "
              f"({busy / a.steps:.2f} ms/step)")
    allbusy = sum(b - a_ for a_, b in union([(s, e) for s, e, _, _ in ks])) / 1e6
    print(f"GPU busy (any queue) {allbusy:.1f} ms = {allbusy / a.steps:.2f} ms/step; idle {span - allbusy:.1f} ms "
          f"= {(span - allbusy) / a.steps:.2f} ms/step")
    lst = sorted(byq[main_q])
    gaps = [((lst[i + 1][0] - lst[i][1]) / 1e3, lst[i][2], lst[i + 1][2]) for i in range(len(lst) - 1)]
    tot = sum(g for g, _, _ in gaps if g > 0) / 1e3
    print(f"main queue: gaps between consecutive kernels {tot:.1f} ms ({tot / a.steps:.2f} ms/step), "
          f"{sum(1 for g, _, _ in gaps if g > 5)} gaps > 5 us")
    def short(name):
        name = name.replace("void ", "").replace("(anonymous namespace)::", "")
        for cut in ("(", "<", " "):
            if cut == "<" and name.startswith("gemm_8ph_kernel"):
                name = name[:name.find(">") + 1] if ">" in name else name
                continue
            i = name.find(cut)
            if i > 0 and not (cut == "<" and "gemm" in name):
                name = name[:i]
        return name[:70]

    hist = defaultdict(float)
    for g, p, n in gaps:
        if g > 0:
            hist[(short(p), short(n))] += g
    for (p, n), g in sorted(hist.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {g / a.steps:8.1f} us/step  {p}  ->  {n}")


if __name__ == "__main__":
    main()
