"""Per-op numerics of the strided convs of tests/test_gpu_no_vendor_conv.py: forward / dgrad / wgrad
of each conv on the native path vs fp32 PyTorch, and per-parameter first-step gradient errors."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_no_vendor_conv import _model  # noqa: E402

from torchbooster_amd.nativize import nativize  # noqa: E402
from torchbooster_amd.ops import conv as CV  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


torch.manual_seed(0)
for (C, K, R, st, pad, H) in [(64, 128, 5, 2, 2, 64), (128, 128, 7, 2, 3, 32), (128, 64, 3, 3, 1, 16), (64, 64, 3, 4, 1, 6)]:
    x = torch.randn(8, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * (C * R * R) ** -0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    xa, wa = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = CV.conv2d(xa, wa, None, st, pad)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pad)
    yr.backward(dy.float())
    print(f"C{C} K{K} {R}x{R}/{st} p{pad} H{H}: fwd {rel(y, yr):.2e} dgrad {rel(xa.grad, xr.grad):.2e} "
          f"wgrad {rel(wa.grad, wr.grad):.2e}", flush=True)
print("routes:", {k: v for k, v in CV.autotune_table().items() if k[0] in ('fwd', 'dgrad', 'wgrad')})
torch.manual_seed(0)
ref = _model().cuda().to(memory_format=torch.channels_last)
m = nativize(copy.deepcopy(ref).to(torch.bfloat16))
x = torch.randn(8, 64, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
t = torch.randint(0, 10, (8,), device="cuda")
F.cross_entropy(ref(x), t).backward()
F.cross_entropy(m(x.to(torch.bfloat16)).float(), t).backward()
ref16 = copy.deepcopy(ref).to(torch.bfloat16)
ref16.zero_grad()
os.environ["TBAMD_FORCE_REFERENCE"] = "1"
F.cross_entropy(ref16(x.to(torch.bfloat16)).float(), t).backward()
for (name, p), pr, p16 in zip(m.named_parameters(), ref.parameters(), ref16.parameters()):
    print(f"{name:12s} native {rel(p.grad, pr.grad):.3e}  stock-bf16 {rel(p16.grad, pr.grad):.3e}")
print(m)
