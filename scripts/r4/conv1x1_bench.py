"""ResNet-50 b256 1x1 convs on the native kernels, as the training step runs them: forward with
the BN-statistics epilogue, and the input gradients with the BN-backward-partial epilogue (BNB 1)
or the residual-add + BN-partial epilogue (ADD 2 + BNB 2).  Prints ms and effective HBM TB/s per
shape (compulsory bytes: operands read once, outputs written once).  Also the 3x3 convs (fwd,
dgrad BNB 1) with TF/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd.ops._ext import native  # noqa: E402

N = int(os.environ.get("B", "256"))
C_ = native()


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def bf(*shape):
    return (torch.randn(*shape, device="cuda") * 0.1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def f32(k, v=None):
    return torch.rand(k, device="cuda") + 0.5 if v is None else torch.full((k,), v, device="cuda")


# (C_in, C_out, H): the bottleneck 1x1 convs of each stage (c1: 4c -> c, c3: c -> 4c)
SH = [(64, 256, 56), (256, 64, 56), (128, 512, 28), (512, 128, 28), (256, 1024, 14), (1024, 256, 14),
      (512, 2048, 7), (2048, 512, 7)]
for Ci, Co, H in SH:
    x = bf(N, Ci, H, H)
    w = bf(Co, Ci, 1, 1)
    px = N * H * H
    ms = t(lambda: C_.conv2d_fwd(x, w, None, 1, 0, False, True))
    gb = px * (Ci + Co) * 2 / 1e9
    r = {"kind": "fwd_stats", "C": Ci, "K": Co, "H": H, "ms": round(ms, 4), "TBs": round(gb / ms, 2)}
    print(json.dumps(r), flush=True)
    # input gradient of this conv: dY [N, Co, H, H] -> dX [N, Ci, H, H] through wt [Ci, Co, 1, 1]
    dy = bf(N, Co, H, H)
    wt = bf(Ci, Co, 1, 1)
    xb = bf(N, Ci, H, H)
    mean, sc, sh = f32(Ci, 0.0), f32(Ci), f32(Ci, 0.0)
    ms1 = t(lambda: C_.conv2d_fwd(dy, wt, None, 1, 0, False, False, None, None, 1, xb, sc, sh, mean, None))
    gb1 = px * (Co + 2 * Ci) * 2 / 1e9
    print(json.dumps({"kind": "dgrad_bnb1", "C": Co, "K": Ci, "H": H, "ms": round(ms1, 4), "TBs": round(gb1 / ms1, 2)}),
          flush=True)
    if Ci > Co:  # the c1 dgrad of a block: + residual gradient (masked) + the previous bn3's partials
        add = bf(N, Ci, H, H)
        amask = torch.randint(0, 256, (px, Ci // 8), device="cuda", dtype=torch.uint8)
        bits = torch.randint(0, 256, (px, Ci // 8), device="cuda", dtype=torch.uint8)
        ms2 = t(lambda: C_.conv2d_fwd(dy, wt, None, 1, 0, False, False, add, amask, 2, xb, None, None, mean, bits))
        gb2 = px * (Co + 3 * Ci) * 2 / 1e9 + 2 * px * Ci / 8 / 1e9
        print(json.dumps({"kind": "dgrad_add2_bnb2", "C": Co, "K": Ci, "H": H, "ms": round(ms2, 4),
                          "TBs": round(gb2 / ms2, 2)}), flush=True)
for c, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
    x = bf(N, c, H, H)
    w = bf(c, c, 3, 3)
    fl = 2 * N * H * H * c * c * 9 / 1e12
    ms = t(lambda: C_.conv2d_fwd(x, w, None, 1, 1, False, True))
    print(json.dumps({"kind": "3x3_fwd_stats", "C": c, "H": H, "ms": round(ms, 4), "TFs": round(fl / ms * 1e3)}),
          flush=True)
    xb = bf(N, c, H, H)
    mean, sc, sh = f32(c, 0.0), f32(c), f32(c, 0.0)
    ms1 = t(lambda: C_.conv2d_fwd(x, w, None, 1, 1, False, False, None, None, 1, xb, sc, sh, mean, None))
    print(json.dumps({"kind": "3x3_dgrad_bnb1", "C": c, "H": H, "ms": round(ms1, 4), "TFs": round(fl / ms1 * 1e3)}),
          flush=True)
