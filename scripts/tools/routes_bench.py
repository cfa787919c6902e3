"""Candidates of the two shapes the shipped route table sent to MIOpen: VGG-19 512@32² bf16 forward
at batch 1 (split-reduction kernel vs the tiled kernel vs MIOpen) and the StyleNet 64 -> 32
upsampling conv's weight gradient (virtual-input MFMA kernel with 32-row dY tiles vs the generic
gather kernel vs MIOpen on the materialised input)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd.ops import conv as CV  # noqa: E402
from torchbooster_amd.ops._ext import native  # noqa: E402

N_ = native()


def t(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return round(s.elapsed_time(e) / reps, 4)


cl = torch.channels_last
for H in (32, 16, 64):
    x = torch.randn(1, 512, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(512, 512, 3, 3, device="cuda") * 0.02).to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(512, device="cuda")
    r = {"shape": f"fwd 1x512x{H}x{H} 3x3 bias bf16",
         "splitk": t(lambda: N_.conv2d_fwd_splitk(x, w, b, 1, 1, False)) if N_.conv_fwd_splitk_ksplit(
             1, 512, 512, 3, 3, H, H) > 1 else None,
         "native": t(lambda: N_.conv2d_fwd(x, w, b, 1, 1, False, False)),
         "miopen": t(lambda: F.conv2d(x, w, b.to(torch.bfloat16), 1, 1))}
    print(json.dumps(r), flush=True)

for (n, h) in ((8, 128), (32, 128)):
    x = torch.randn(n, 64, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(n, 32, 2 * h, 2 * h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn(32, 64, 3, 3, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)

    def mio():
        xv = CV._virtual(x, 1, 2, True).contiguous(memory_format=cl)
        return CV._miopen_bwd(dy, xv, w, 1, 0, 1)

    r = {"shape": f"wgrad {n}x64x{h}x{h} up2 reflect -> 32x64x3x3 bf16",
         "virt32": t(lambda: N_.conv2d_wgrad_virtual(dy, x, 3, 3, 1, 1, 2, True)),
         "any": t(lambda: N_.conv_any_wgrad(dy, x, 3, 3, 1, 1, 2, True)),
         "miopen": t(mio)}
    print(json.dumps(r), flush=True)
