"""In-context check of every forward conv of a ResNet-50 step under the big-tile heuristic: each call
is recomputed on the same tensors with the 128x128 kernels, and its statistics rows are checked
against sums of its own output."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from torchbooster_amd import models
from torchbooster_amd.ops import conv as CV
from torchbooster_amd.ops._ext import native

C = native()
orig = CV._fwd
rep = []


def patched(x, w, bias, stride, pad, want_stats, relu=False, fold=None):
    out = orig(x, w, bias, stride, pad, want_stats, relu, fold)
    y, st = out[0], out[1]
    mode = C.conv_get_big()
    C.conv_set_big(0)
    y0, st0 = C.conv2d_fwd(x, w, bias, stride, pad, relu, want_stats)
    C.conv_set_big(mode)
    torch.cuda.synchronize()
    dy = (y.float() - y0.float()).abs().max().item()
    msg = f"{tuple(x.shape)} w{tuple(w.shape)} s{stride} p{pad} stats={want_stats} y-diff {dy:.3g}"
    if want_stats and st is not None:
        K = y.shape[1]
        yf = y.permute(0, 2, 3, 1).reshape(-1, K).double()
        own = st.double().sum(0)
        ref = torch.stack([yf.sum(0), (yf * yf).sum(0)])
        e = ((own - ref).abs().max() / ref.abs().max()).item()
        e0 = ((st0.double().sum(0) - ref).abs().max() / ref.abs().max()).item()
        msg += f" rows {st.shape[0]}/{st0.shape[0]} stats-err big {e:.3g} old {e0:.3g}"
    rep.append(msg)
    return out


CV._fwd = patched
C.conv_set_big(1)
torch.manual_seed(0)
m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
x = torch.randn(8, 3, 96, 96, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
m(x)
torch.cuda.synchronize()
for r in rep:
    print(r)
