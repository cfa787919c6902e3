"""Communication / compute overlap in a rocprofv3 kernel trace.

Usage: python scripts/overlap.py run_kernel_trace.csv [--marker adamw_mt] [--last 2]

For the last K steps (delimited by the optimizer kernel) prints, for every RCCL
kernel, its queue, duration and how much of it ran while a compute kernel on
another queue was executing -- the evidence that the reducer's bucket
all-reduces overlap backward rather than serialise behind it.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_mt")
    ap.add_argument("--last", type=int, default=2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["q"] = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    rows.sort(key=lambda r: r["s"])
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo = marks[-a.last - 1] + 1 if len(marks) > a.last else 0
    hi = marks[-1] + 1 if marks else len(rows)
    sel = rows[lo:hi]
    comm = [r for r in sel if any(t in r["Kernel_Name"].lower() for t in ("nccl", "rccl", "onerankreduce"))]
    comp = [r for r in sel if r not in comm]
    t0 = sel[0]["s"] if sel else 0
    tot, ovl = 0, 0
    print(f"{len(comm)} RCCL kernels over the last {a.last} steps")
    for c in comm:
        d = c["e"] - c["s"]
        o = 0
        cover = sorted((max(c["s"], k["s"]), min(c["e"], k["e"])) for k in comp
                       if k["q"] != c["q"] and k["s"] < c["e"] and k["e"] > c["s"])
        cur = c["s"]
        for s, e in cover:  # union of the overlapping compute intervals
            s = max(s, cur)
            if e > s:
                o += e - s
                cur = e
        tot += d
        ovl += o
        print(f"  t={(c['s'] - t0) / 1e3:9.1f} us  q={c['q']:>3}  {d / 1e3:7.1f} us  overlapped {o / 1e3:7.1f} us"
              f"  {c['Kernel_Name'][:70]}")
    if tot:
        print(f"total RCCL {tot / 1e3:.1f} us, {100.0 * ovl / tot:.1f} % of it concurrent with compute on other queues")
    qs = sorted({r['q'] for r in comp})
    print("compute queues:", qs)


if __name__ == "__main__":
    main()
