"""Every conv2d_fwd call of a ResNet-50 training step (forward + input-gradient forms) under the
big-tile heuristic, recomputed in context with the 128x128 kernels on the same tensors."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from torchbooster_amd import models
from torchbooster_amd.ops._ext import native

C = native()
orig = C.conv2d_fwd
rep = []


def patched(*a, **k):
    out = orig(*a, **k)
    mode = C.conv_get_big()
    C.conv_set_big(0)
    ref = orig(*a, **k)
    C.conv_set_big(mode)
    torch.cuda.synchronize()
    dy = (out[0].float() - ref[0].float()).abs().max().item()
    msg = f"{tuple(a[0].shape)} w{tuple(a[1].shape)} bnb={k.get('bnb_mode', a[9] if len(a) > 9 else 0)} " \
          f"add={'addend' in k or (len(a) > 7 and a[7] is not None)} y-diff {dy:.3g}"
    if len(out) > 1 and out[1] is not None and out[1].dim() == 3:
        s1, s0 = out[1].double().sum(0), ref[1].double().sum(0)
        msg += f" aux rows {out[1].shape[0]}/{ref[1].shape[0]} aux-diff {((s1 - s0).abs().max() / s0.abs().max()).item():.3g}"
    rep.append(msg)
    return out


C.conv2d_fwd = patched
C.conv_set_big(1)
torch.manual_seed(0)
m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
x = torch.randn(8, 3, 96, 96, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
m(x).float().square().mean().backward()
torch.cuda.synchronize()
for r in rep:
    print(r)
