"""Is the mismatch split-related or history-related?  ref = 2nd split-off run; then alternate
off / on / on-with-synced-wgrad runs and report each run's worst relative gradient difference."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("TB_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.ops import conv as convmod  # noqa: E402
from torchbooster_amd.ops import streams  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

_orig = convmod._wgrad
SYNC = [False]


def _wgrad_synced(*a, **k):
    r = _orig(*a, **k)
    if SYNC[0]:
        torch.cuda.current_stream().synchronize()
    return r


convmod._wgrad = _wgrad_synced


def run(split, steps=2, sync=False):
    streams.set_enabled(split)
    SYNC[0] = sync
    torch.manual_seed(0)
    m = models.resnet18(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    g = torch.Generator(device="cuda").manual_seed(1)
    out = []
    for _ in range(steps):
        x = torch.randn(16, 3, 64, 64, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 10, (16,), device="cuda", generator=g)
        opt.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(m(x).float(), y).backward()
        torch.cuda.synchronize()
        out.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
        opt.step()
    streams.set_enabled(True)
    SYNC[0] = False
    return out


def worst(got, ref):
    r = []
    for s in range(len(ref)):
        v = max(((got[s][n].float() - ref[s][n].float()).norm().item() / (ref[s][n].float().norm().item() + 1e-12), n)
                for n in ref[s])
        r.append((round(v[0], 5), v[1]))
    return r


run(False)
ref = run(False)
for i in range(3):
    for name, kw in (("off", dict(split=False)), ("on", dict(split=True)), ("on+sync", dict(split=True, sync=True))):
        print(i, name, worst(run(**kw), ref), flush=True)
