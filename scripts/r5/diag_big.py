"""Layer-by-layer comparison of the ResNet-50 training step with the big-tile conv (TBAMD_CONV_BIG
heuristic) against the 128x128 kernels: logits, BN running statistics after the forward, and every
parameter gradient; prints the worst offenders of each kind."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from torchbooster_amd import models
from torchbooster_amd.ops._ext import native

C = native()


def run(mode, H=64, B=4):
    C.conv_set_big(mode)
    torch.manual_seed(0)
    m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    x = torch.randn(B, 3, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    acts = {}
    hooks = []
    for n, mod in m.named_modules():
        if n.count(".") == 1 and n.startswith("layer"):
            hooks.append(mod.register_forward_hook(lambda mod, i, o, n=n: acts.__setitem__(n, o.float().clone())))
    out = m(x)
    logits = out.float().clone()
    rs = {n: b.float().clone() for n, b in m.named_buffers() if "running" in n}
    out.float().square().mean().backward()
    torch.cuda.synchronize()
    g = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    for h in hooks:
        h.remove()
    return logits, acts, rs, g


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


H = int(sys.argv[1]) if len(sys.argv) > 1 else 64
run(0, H)
l0, a0, r0, g0 = run(0, H)
l0b, a0b, r0b, g0b = run(0, H)
l1, a1, r1, g1 = run(1, H)
print("logits rerun", rel(l0b, l0), "big", rel(l1, l0))
for n in a0:
    print(f"act {n:12s} rerun {rel(a0b[n], a0[n]):.3e} big {rel(a1[n], a0[n]):.3e}")
print("running-mean deviation in model order (first nonzero = where the paths diverge):")
for n in r0:
    if n.endswith("running_mean"):
        print(f"  {n:36s} big {rel(r1[n], r0[n]):.3e} rerun {rel(r0b[n], r0[n]):.3e}")
wg = sorted(((rel(g1[n], g0[n]), rel(g0b[n], g0[n]), n) for n in g0), reverse=True)[:16]
print("grads worst (big, rerun):")
for a, b, n in wg:
    print(f"  {a:.3e} {b:.3e} {n}")
# every conv weight grad
print("conv grads big-vs-rerun ratio (first 20 by name):")
for n in [n for n in g0 if "conv.weight" in n][:20]:
    print(f"  {n:28s} big {rel(g1[n], g0[n]):.3e} rerun {rel(g0b[n], g0[n]):.3e}")
