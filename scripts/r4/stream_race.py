"""Hunt the intermittent side-stream gradient mismatch (tests/test_gpu_streams.py): one process,
split off as the reference, then many split-on runs; prints every run whose gradients differ."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("TB_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.ops import streams  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402


def run(split, steps=2):
    streams.set_enabled(split)
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
        out.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
        opt.step()
    streams.set_enabled(True)
    return out


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


run(False)
ref = run(False)
bad = 0
N = int(os.environ.get("N", "30"))
for i in range(N):
    got = run(True)
    for s in range(len(ref)):
        worst = sorted(((rel(got[s][n], ref[s][n]), n) for n in ref[s]), reverse=True)[:3]
        if worst[0][0] > 1e-3:
            bad += 1
            print(f"run {i} step {s}: {[(round(v, 4), n) for v, n in worst]}", flush=True)
print(f"stop_events={os.environ.get('TBAMD_STOP_EVENTS', '1')} bad={bad}/{N}", flush=True)
