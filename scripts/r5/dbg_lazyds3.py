"""Debug: per-block forward outputs of ResNet-50 (b4, 64 px) with the lazy affine downsample on/off."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.models import resnet as R  # noqa: E402

torch.manual_seed(0)
model = R.resnet50(num_classes=16).cuda().to(torch.bfloat16).train()
x0 = torch.randn(4, 3, 64, 64, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
outs = {}
for lazy in (False, True):
    R._LAZY_DS = lazy
    R._RES_CARRIER = True
    p = model.pool
    x = model.stem(x0, pool=(p.kernel_size, p.stride, p.padding))
    link = None
    for si, stage in enumerate((model.layer1, model.layer2, model.layer3, model.layer4)):
        for bi, blk in enumerate(stage):
            x, link = blk.forward_linked(x, link)
            outs.setdefault((si, bi), []).append(x.detach().float().clone())
rel = lambda u, v: ((u - v).norm() / v.norm().clamp_min(1e-12)).item()
for n, (a, b) in outs.items():
    print(n, tuple(a.shape), "%.5f" % rel(b, a))
