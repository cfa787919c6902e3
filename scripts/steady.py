"""Steady-state per-step kernel table from a rocprofv3 kernel_trace.csv.

Steps are delimited by the optimizer launch (adamw_mt_k / sgd_mt_k, or the
stock multi_tensor_apply / foreach AdamW kernels); the last ``nsteps`` steps are
summarised.  ``per_step`` optimizer launches form one training step (e.g. 2 for
a G/D GAN step)."""
import collections
import csv
import re
import sys


def main(path, nsteps=3, per_step=1, top=30):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if re.search(r"adamw_mt_k|sgd_mt_k|multi_tensor_apply_kernel|FusedAdam", r["Kernel_Name"])]
    # collapse consecutive optimizer launches of one step
    ends = []
    for i in opt:
        if not ends or i - ends[-1] > 3:
            ends.append(i)
        else:
            ends[-1] = i
    ends = ends[::per_step] if per_step > 1 else ends
    a, b = ends[-1 - nsteps], ends[-1]
    sel = rows[a + 1: b + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += d
    busy = sum(v[1] for v in agg.values()) / nsteps
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / nsteps
    print(f"steady state over {nsteps} steps: wall {wall:.3f} ms/step, kernel busy {busy:.3f} ms/step, "
          f"{len(sel) / nsteps:.0f} dispatches/step")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / nsteps:8.3f} ms {n / nsteps:5.1f}x  {k[:140]}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(v) for v in sys.argv[2:]))
