"""Uninitialised-memory hunt: every at::empty / torch.empty is NaN-filled (deterministic mode
fill); any gradient that picks up a NaN read an unwritten workspace row."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("TB_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

t = torch.empty(8, device="cuda")
print("empty is NaN-filled:", bool(torch.isnan(t).all()), flush=True)
name = os.environ.get("MODEL", "resnet18")
for trial in range(2):
    torch.manual_seed(0)
    m = getattr(models, name)(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    for step in range(3):
        x = torch.randn(16, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (16,), device="cuda")
        opt.zero_grad(set_to_none=True)
        out = m(x)
        if not torch.isfinite(out).all():
            print(f"trial {trial} step {step}: non-finite forward output", flush=True)
        torch.nn.functional.cross_entropy(out.float(), y).backward()
        torch.cuda.synchronize()
        badp = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        print(f"trial {trial} step {step}: {len(badp)} params with non-finite grads {badp[:8]}", flush=True)
        opt.step()
