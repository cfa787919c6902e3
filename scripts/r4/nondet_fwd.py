"""First module whose forward output differs between two post-tuning forwards of the same
native ResNet on the same input (module forward hooks, execution order)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd import models  # noqa: E402

name = os.environ.get("MODEL", "resnet18")
torch.manual_seed(0)
m = getattr(models, name)(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
m.train()
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randn(16, 3, 64, 64, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
rec = []


def hook(mod, inp, out, nm=None):
    outs = out if isinstance(out, (tuple, list)) else (out,)
    rec.append((nm, [o.detach().clone() for o in outs if torch.is_tensor(o)]))


for n, mod in m.named_modules():
    if n:
        mod.register_forward_hook(lambda mod, i, o, nm=n: hook(mod, i, o, nm))
state = {k: v.clone() for k, v in m.state_dict().items()}
runs = []
for r in range(4):
    m.load_state_dict(state)
    rec.clear()
    with torch.no_grad():
        m(x)
    torch.cuda.synchronize()
    runs.append(list(rec))
for r in (2, 3):
    first = None
    for (n1, o1), (n2, o2) in zip(runs[1], runs[r]):
        for a, b in zip(o1, o2):
            if not torch.equal(a, b):
                d = (a.float() - b.float()).abs()
                first = (n1, d.max().item(), int((d > 0).sum()), tuple(a.shape))
                break
        if first:
            break
    print(f"run 1 vs {r}: first differing module {first}", flush=True)
