"""Per-kernel summary of the steady-state steps in a rocprofv3 rocpd database.

usage: python scripts/dbstats.py <run_results.db> [--steps K] [--marker REGEX] [--top N]

Step boundaries are the dispatches whose name matches --marker (default: the fused
AdamW kernel, which ends every training step); the last K complete steps are
aggregated (per-step averages) and printed sorted by time.
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default=r"adamw_mt_k")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--markers-per-step", type=int, default=1, help="e.g. 2 for a G+D step with two optimizers")
    ap.add_argument("--width", type=int, default=90)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    mk = re.compile(a.marker)
    ends = []
    for i, (n, s, e) in enumerate(rows):
        if mk.search(n) and (not ends or i > ends[-1] + 1):
            ends.append(i)
        elif mk.search(n):
            ends[-1] = i
    ends = ends[len(ends) % a.markers_per_step:][a.markers_per_step - 1::a.markers_per_step]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} step markers")
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    seg = rows[lo:hi]
    agg = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for n, s, e in seg:
        n = re.sub(r"^void ", "", n)
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
        busy += (e - s) / 1e6
    wall = (seg[-1][2] - seg[0][1]) / 1e6
    K = a.steps
    print(f"steps={K} dispatches/step={len(seg) // K} kernel-busy ms/step={busy / K:.3f} "
          f"wall ms/step={wall / K:.3f}")
    print(f"{'kernel':{a.width}s} {'calls':>6s} {'ms':>8s} {'%':>6s}")
    for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{n[: a.width]:{a.width}s} {cnt / K:6.1f} {t / K:8.3f} {100 * t / busy:6.1f}")


if __name__ == "__main__":
    main()
