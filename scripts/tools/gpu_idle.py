"""Whole-GPU idle time in a steady-state step of a rocprofv3 kernel trace: intervals where NO stream
runs a kernel, with the kernels around each (what the critical path waits for), plus each stream's
busy time.  python scripts/tools/gpu_idle.py TRACE.csv [nsteps=3] [marker=adamw_mt_k]"""
import csv
import re
import sys


def short(n, k=60):
    n = re.sub(r"tbamd::|\(anonymous namespace\)::|void |at::native::", "", n)
    return re.sub(r"\(.*", "", n)[:k]


def main(path, nsteps=3, marker="adamw_mt_k"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if re.search(marker, r["Kernel_Name"])]
    ends = []
    for i in opt:
        if not ends or i - ends[-1] > 3:
            ends.append(i)
        else:
            ends[-1] = i
    a, b = ends[-1 - nsteps], ends[-1]
    sel = rows[a + 1: b + 1]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in sel)
    gaps, cur_end, prev = [], t0, None
    for s, e, r in iv:
        if s > cur_end and prev is not None:
            gaps.append((s - cur_end, prev, r))
        if e > cur_end:
            cur_end, prev = e, r
    idle = sum(g for g, _, _ in gaps)
    wall = (t1 - t0) / nsteps / 1e6
    print(f"{nsteps} steps, wall {wall:.3f} ms/step, whole-GPU idle {idle / nsteps / 1e6:.3f} ms/step "
          f"({len(gaps) / nsteps:.0f} gaps/step)")
    for g, p, r in sorted(gaps, key=lambda x: -x[0])[:25]:
        print(f"  {g / 1e3:8.1f} us  {short(p['Kernel_Name'])} -> {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(v) if v.isdigit() else v for v in sys.argv[2:]))
