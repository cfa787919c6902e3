"""Run an example with ATen GEMM / conv entry points wrapped: every call on a CUDA tensor is
counted with its caller (file:line chain), to find which code path still reaches hipBLASLt /
MIOpen.  usage: python scripts/r3/blas_spy.py examples/img_cls/lenet/lenet.py"""
import atexit
import collections
import runpy
import sys
import traceback

import torch
import torch.nn.functional as F

CALLS = collections.Counter()


def _wrap(owner, name):
    fn = getattr(owner, name)

    def w(*a, **k):
        if any(isinstance(t, torch.Tensor) and t.is_cuda for t in a):
            st = [f"{f.filename.split('/repo/')[-1]}:{f.lineno}" for f in traceback.extract_stack()[:-1]
                  if "site-packages" not in f.filename][-4:]
            shapes = tuple(tuple(t.shape) for t in a if isinstance(t, torch.Tensor))
            CALLS[(name, str(shapes), " <- ".join(reversed(st)))] += 1
        return fn(*a, **k)

    setattr(owner, name, w)


for n in ("linear", "conv2d", "conv_transpose2d"):
    _wrap(F, n)
for n in ("mm", "addmm", "matmul", "bmm", "baddbmm"):
    _wrap(torch, n)
_orig_matmul = torch.Tensor.__matmul__


def _mm(self, other):
    if self.is_cuda:
        st = [f"{f.filename.split('/repo/')[-1]}:{f.lineno}" for f in traceback.extract_stack()[:-1]
              if "site-packages" not in f.filename][-4:]
        CALLS[("@", str((tuple(self.shape), tuple(other.shape))), " <- ".join(reversed(st)))] += 1
    return _orig_matmul(self, other)


torch.Tensor.__matmul__ = _mm


@atexit.register
def _report():
    for (n, s, st), c in CALLS.most_common(40):
        print(f"[blas-spy] {c:5d} {n} {s} {st}", file=sys.stderr, flush=True)


path = sys.argv[1]
sys.argv = sys.argv[1:]
runpy.run_path(path, run_name="__main__")
