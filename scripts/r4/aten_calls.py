"""Which layers of a workload's steady-state step still call ATen's library-backed ops
(F.conv2d / conv_transpose2d / linear / addmm / mm / matmul -> MIOpen / hipBLASLt)?  Runs the
bench_workloads step a few times, then records the Python call sites of those ops for 2 steps."""
import collections
import os
import sys
import traceback

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "scripts"))

HITS = collections.Counter()
REC = [False]


def wrap(mod, name):
    orig = getattr(mod, name)

    def f(*a, **k):
        if REC[0]:
            st = [fr for fr in traceback.extract_stack()[:-1] if "torchbooster_amd" in fr.filename or "bench_workloads" in fr.filename]
            where = " <- ".join(f"{os.path.basename(fr.filename)}:{fr.lineno}" for fr in st[-3:])
            shapes = tuple(tuple(x.shape) for x in a if isinstance(x, torch.Tensor))
            HITS[(name, shapes, where)] += 1
        return orig(*a, **k)

    setattr(mod, name, f)


for n in ("conv2d", "conv_transpose2d", "linear"):
    wrap(F, n)
for n in ("addmm", "mm", "matmul", "bmm", "conv2d"):
    wrap(torch, n)

import bench_workloads as BW  # noqa: E402
from torchbooster_amd.ops import conv as CV  # noqa: E402

_time_ms = CV._time_ms


def timed(fn, *a, **k):  # a conv route being timed inside the recorded steps = first-use tuning
    if REC[0]:
        st = [fr for fr in traceback.extract_stack()[:-1] if "torchbooster_amd" in fr.filename]
        HITS[("conv-tuning", (), " <- ".join(f"{os.path.basename(fr.filename)}:{fr.lineno}" for fr in st[-3:]))] += 1
    return _time_ms(fn, *a, **k)


CV._time_ms = timed

wl = sys.argv[1] if len(sys.argv) > 1 else "dcgan"


def timeit(step, warmup, steps):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    REC[0] = True
    out = None
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    REC[0] = False
    return 1.0, out


BW._timeit = timeit
sys.argv = [sys.argv[0], "--workload", wl, "--mode", "native", "--steps", "3", "--warmup", "6"] + sys.argv[2:]
try:
    BW.main()
except SystemExit:
    pass
print(f"ATen library-op calls / route timings in 3 steady-state steps: {sum(HITS.values())}")
for (n, s, w), c in HITS.most_common(40):
    print(f"{c:4d}  {n}{s}  {w}")
