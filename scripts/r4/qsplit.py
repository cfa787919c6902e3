"""Per-queue busy time of the steady-state steps of a rocprofv3 kernel trace.

Usage: python scripts/r4/qsplit.py kernel_trace.csv [--marker stem_pad_k] [--last 3]
Prints, per HIP queue, the busy time per step (union of kernel intervals), the kernels that take
most of it, and the idle gaps of the busiest (compute) queue."""
import argparse
import csv
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def short(n):
    n = n.replace("tbamd::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="stem_pad_k")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = marks[-a.last - 1], marks[-1]
    sel = rows[lo:hi]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(rows[hi]["Start_Timestamp"])
    wall = (t1 - t0) / a.last / 1e6
    byq = defaultdict(list)
    for r in sel:
        byq[r["Queue_Id"]].append(r)
    print(f"{a.last} steps, wall {wall:.3f} ms/step")
    for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        busy = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]) / a.last / 1e6
        agg = defaultdict(lambda: [0.0, 0])
        for r in rs:
            k = agg[short(r["Kernel_Name"])]
            k[0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / a.last / 1e6
            k[1] += 1
        print(f"queue {q}: {len(rs) // a.last} dispatches/step, busy {busy:.3f} ms/step")
        for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
            print(f"   {t:7.3f} ms {c / a.last:5.1f}x  {n}")
    # gaps on the busiest queue
    q = max(byq, key=lambda k: len(byq[k]))
    rs = sorted(byq[q], key=lambda r: int(r["Start_Timestamp"]))
    gaps = []
    for p, n in zip(rs, rs[1:]):
        g = int(n["Start_Timestamp"]) - int(p["End_Timestamp"])
        if g > 0:
            gaps.append((g, short(p["Kernel_Name"]), short(n["Kernel_Name"])))
    tg = sum(g for g, _, _ in gaps) / a.last / 1e6
    print(f"queue {q} idle gaps: {tg:.3f} ms/step over {len(gaps) // a.last} gaps/step; largest:")
    for g, p, n in sorted(gaps, reverse=True)[:10]:
        print(f"   {g / 1e3:8.1f} us  after {p[:60]}  before {n[:60]}")


if __name__ == "__main__":
    main()
