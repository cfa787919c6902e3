"""Debug: one downsample bottleneck, lazy affine downsample output on/off: forward output and grads."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.models import resnet as R  # noqa: E402

torch.manual_seed(0)
blk = R.Bottleneck(64, 64, 1).cuda().to(torch.bfloat16).train()
x = torch.randn(4, 64, 16, 16, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
res = {}
for lazy in (False, True):
    R._LAZY_DS = lazy
    R._RES_CARRIER = True
    blk.zero_grad(set_to_none=True)
    xi = x.detach().clone().requires_grad_()
    out, _ = blk.forward_linked(xi)
    out.float().square().mean().backward()
    res[lazy] = (out.detach().float(), xi.grad.float(), {n: p.grad.float() for n, p in blk.named_parameters()})
a, b = res[False], res[True]
rel = lambda u, v: ((u - v).norm() / v.norm().clamp_min(1e-12)).item()
print("out", rel(b[0], a[0]), "dx", rel(b[1], a[1]))
for n in a[2]:
    print(n, rel(b[2][n], a[2][n]))
