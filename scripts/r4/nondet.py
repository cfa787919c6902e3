"""Localise run-to-run nondeterminism of the native ResNet-18 step: the same seed/data twice
(fresh models), comparing logits, loss and every gradient of step 0."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

name = os.environ.get("MODEL", "resnet18")


def run():
    torch.manual_seed(0)
    m = getattr(models, name)(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(16, 3, 64, 64, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda", generator=g)
    w0 = {n: p.detach().clone() for n, p in m.named_parameters()}
    logits = m(x)
    loss = torch.nn.functional.cross_entropy(logits.float(), y)
    loss.backward()
    torch.cuda.synchronize()
    bufs = {n: b.detach().clone() for n, b in m.named_buffers()}
    return w0, logits.detach().clone(), float(loss), {n: p.grad.detach().clone() for n, p in m.named_parameters()}, bufs


runs = [run() for _ in range(4)]
for i in range(1, 4):
    w, l, ls, gr, bf = runs[i]
    w0, l0, ls0, gr0, bf0 = runs[0]
    wd = max((w[n].float() - w0[n].float()).abs().max().item() for n in w)
    ld = (l.float() - l0.float()).abs().max().item()
    bd = sorted((((bf[n].float() - bf0[n].float()).abs().max().item()), n) for n in bf)[-3:]
    gd = sorted((((gr[n].float() - gr0[n].float()).norm() / (gr0[n].float().norm() + 1e-12)).item(), n) for n in gr)[-5:]
    print(f"run {i}: init diff {wd:.3g} logits diff {ld:.3g} loss {ls:.6f} vs {ls0:.6f}", flush=True)
    print(f"   buffers worst {[(round(v, 5), n) for v, n in bd]}", flush=True)
    print(f"   grads worst {[(round(v, 5), n) for v, n in gd]}", flush=True)
