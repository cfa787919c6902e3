"""Per-kernel stats from a rocprofv3 kernel_trace.csv restricted to the steady state.

Usage: python scripts/ktrace.py run_kernel_trace.csv|run_results.db --marker <substr> --last K [--top N]
Steps are delimited by occurrences of a kernel whose name contains --marker
(e.g. the optimizer kernel 'adamw_mt'); the last K steps are summarised.
"""
import argparse
import csv
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kstats import CATS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_mt")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocprofv3 default (rocpd sqlite) output
        import sqlite3

        con = sqlite3.connect(a.trace)
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.last + 1:
        print("not enough steps", len(marks))
        return
    lo, hi = marks[-a.last - 1] + 1, marks[-1] + 1
    sel = rows[lo:hi]
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / a.last
    per = defaultdict(lambda: [0, 0.0])
    cat = defaultdict(float)
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        busy += d
        per[r["Kernel_Name"]][0] += 1
        per[r["Kernel_Name"]][1] += d
        for c, pat in CATS:
            if re.search(pat, r["Kernel_Name"]):
                break
        else:
            c = "other"
        cat[c] += d
    print(f"steady state over {a.last} steps: wall {wall:.2f} ms/step, kernel busy {busy / a.last:.2f} ms/step, "
          f"{len(sel) // a.last} dispatches/step")
    for c, t in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"  {c:14s} {t / a.last:8.2f} ms/step")
    print("top kernels (ms/step, calls/step):")
    for k, (n, t) in sorted(per.items(), key=lambda x: -x[1][1])[: a.top]:
        print(f"  {t / a.last:7.3f} {n // a.last:4d}  {k[:120]}")


if __name__ == "__main__":
    main()
