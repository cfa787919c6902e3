"""ResNet-50 b256 conv weight gradients on the native split-K kernel + its reduce, in isolation
(one stream, no concurrent compute): ms and TF/s per shape.  Run under TBAMD_WGRAD_WAVES=f to see
the split count's effect (fewer splits = fewer partial bytes for the reduce)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd.ops._ext import native  # noqa: E402

N = int(os.environ.get("B", "256"))
C_ = native()


def t(fn, reps=10):
    for _ in range(2):
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


# (C_in, C_out, R, H_out, stride)
SH = [(64, 64, 1, 56, 1), (64, 64, 3, 56, 1), (64, 256, 1, 56, 1), (256, 64, 1, 56, 1), (128, 128, 3, 28, 1),
      (128, 512, 1, 28, 1), (512, 128, 1, 28, 1), (256, 256, 3, 14, 1), (256, 1024, 1, 14, 1), (1024, 256, 1, 14, 1),
      (512, 512, 3, 7, 1), (512, 2048, 1, 7, 1), (2048, 512, 1, 7, 1), (256, 512, 1, 28, 2), (128, 128, 3, 28, 2)]
tot = 0.0
for C, K, R, H, st in SH:
    Hin = H * st
    x = bf(N, C, Hin, Hin)
    dy = bf(N, K, H, H)
    pad = R // 2
    ms = t(lambda: C_.conv2d_wgrad(dy, x, R, R, st, pad))
    fl = 2 * N * H * H * K * C * R * R / 1e12
    tot += ms
    print(json.dumps({"C": C, "K": K, "R": R, "H": H, "stride": st, "ms": round(ms, 4), "TFs": round(fl / ms * 1e3)}),
          flush=True)
print(json.dumps({"total_ms": round(tot, 3)}), flush=True)
