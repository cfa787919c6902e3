"""Main-stream timeline of the steady-state training step from a rocprofv3 kernel_trace.csv: per
stream busy / idle time, the main stream's kernel classes, its largest idle gaps (with the kernels
around them) and the per-call durations of a chosen kernel.

python scripts/tools/critpath.py TRACE.csv [nsteps=3] [kernel-regex=colsum_fin4]"""
import collections
import csv
import re
import sys


def short(name, n=70):
    name = re.sub(r"tbamd::|\(anonymous namespace\)::|void ", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:n]


def main(path, nsteps=3, pat="colsum_fin4"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if re.search(r"adamw_mt_k|sgd_mt_k", r["Kernel_Name"])]
    ends = []
    for i in opt:
        if not ends or i - ends[-1] > 3:
            ends.append(i)
        else:
            ends[-1] = i
    a, b = ends[-1 - nsteps], ends[-1]
    sel = rows[a + 1: b + 1]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    skey = "Stream_Id" if "Stream_Id" in sel[0] else "Queue_Id"
    by = collections.defaultdict(list)
    for r in sel:
        by[r[skey]].append(r)
    main_s = max(by, key=lambda s: len(by[s]))
    wall = (t1 - t0) / 1e6 / nsteps
    print(f"{nsteps} steps, wall {wall:.3f} ms/step; streams by {skey}:")
    for s, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e6 / nsteps
        print(f"  {s}: {len(rs) / nsteps:.0f} dispatches/step, busy {busy:.3f} ms/step{'  (main)' if s == main_s else ''}")
    ms = by[main_s]
    cls = collections.defaultdict(lambda: [0, 0.0])
    gaps = []
    prev = None
    idle = 0.0
    for r in ms:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        cls[short(r["Kernel_Name"], 40)][0] += 1
        cls[short(r["Kernel_Name"], 40)][1] += (e - s) / 1e6
        if prev is not None:
            g = (s - int(prev["End_Timestamp"])) / 1e6
            if g > 0:
                idle += g
                gaps.append((g, short(prev["Kernel_Name"], 50), short(r["Kernel_Name"], 50)))
        prev = r
    print(f"main stream: busy {sum(v[1] for v in cls.values()) / nsteps:.3f} ms/step, idle {idle / nsteps:.3f} ms/step "
          f"({len(gaps) / nsteps:.0f} gaps/step, median {sorted(g[0] for g in gaps)[len(gaps) // 2] * 1e3:.1f} us)")
    for k, (n, t) in sorted(cls.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {t / nsteps:7.3f} ms {n / nsteps:5.1f}x  {k}")
    print("largest main-stream gaps (us, after -> before):")
    for g, p, n in sorted(gaps, reverse=True)[:15]:
        print(f"  {g * 1e3:8.1f}  {p} -> {n}")
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ms if re.search(pat, r["Kernel_Name"])]
    if durs:
        durs.sort()
        n = len(durs)
        print(f"{pat}: {n / nsteps:.0f}/step, us min {durs[0]:.1f} p25 {durs[n // 4]:.1f} med {durs[n // 2]:.1f} "
              f"p75 {durs[3 * n // 4]:.1f} max {durs[-1]:.1f}, sum {sum(durs) / nsteps / 1e3:.3f} ms/step")
        seq = [(short(r["Kernel_Name"], 40), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
               for r in ms[: len(ms) // nsteps]]
        for i, (k, d) in enumerate(seq):
            if re.search(pat, k):
                print(f"  #{i:3d} {d:7.1f} us  after {seq[i - 1][0]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3, sys.argv[3] if len(sys.argv) > 3 else "colsum_fin4")
