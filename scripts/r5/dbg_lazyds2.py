"""Debug: ResNet-50 (b4, 64 px), lazy affine downsample on/off (carrier on in both): logits and grads."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.models import resnet as R  # noqa: E402

torch.manual_seed(0)
model = R.resnet50(num_classes=16).cuda().to(torch.bfloat16).train()
x = torch.randn(4, 3, 64, 64, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
res = {}
for lazy in (False, True, False):
    R._LAZY_DS = lazy
    R._RES_CARRIER = True
    model.zero_grad(set_to_none=True)
    out = model(x).float()
    out.square().mean().backward()
    res.setdefault(lazy, []).append((out.detach(), {n: p.grad.float().clone() for n, p in model.named_parameters()}))
rel = lambda u, v: ((u - v).norm() / v.norm().clamp_min(1e-12)).item()
a, b, a2 = res[False][0], res[True][0], res[False][1]
print("logits lazy vs off", rel(b[0], a[0]), " off vs off", rel(a2[0], a[0]))
bad = [(n, rel(b[1][n], a[1][n]), rel(a2[1][n], a[1][n])) for n in a[1]]
for n, d, d0 in bad[:6] + [t for t in bad if t[1] > 0.05][:20]:
    print(f"{n:40s} lazy {d:.4f}  rerun {d0:.4f}")
