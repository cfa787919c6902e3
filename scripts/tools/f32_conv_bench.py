"""fp32 3x3 convs of the style-transfer examples (VGG-19 relu1-4 at 256 px batch 8, StyleNet):
native generic conv in split-bf16 / exact-f32 MFMA mode vs MIOpen fp32, fwd / dgrad / wgrad."""
import json
import torch
import torch.nn.functional as F
from torchbooster_amd.ops._ext import native

SH = [(8, 3, 256, 64), (8, 64, 256, 64), (8, 64, 128, 128), (8, 128, 128, 128), (8, 128, 64, 256),
      (8, 256, 64, 256), (8, 256, 32, 512), (8, 512, 32, 512), (8, 128, 64, 128)]


def t(fn, reps=10):
    fn(); fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps):
        fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps


C_ = native()
for N, C, H, K in SH:
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, device="cuda") / (9 * C) ** 0.5).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    r = {"shape": [N, C, H, K]}
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = F.conv2d(xr, wr, None, 1, 1)
    yr.backward(dy)
    for mode in ("split", "exact"):
        C_.conv_any_set_f32_split(mode == "split")
        r[f"fwd_{mode}"] = t(lambda: C_.conv_any_fwd(x, w, None, 1, 1, 1, False))
        r[f"dgrad_{mode}"] = t(lambda: C_.conv_any_dgrad(dy, w, H, H, 1, 1, 1, False))
        r[f"wgrad_{mode}"] = t(lambda: C_.conv_any_wgrad(dy, x, 3, 3, 1, 1, 1, False))
        y = C_.conv_any_fwd(x, w, None, 1, 1, 1, False)
        r[f"err_{mode}"] = ((y - yr).norm() / yr.norm()).item()
        dw = C_.conv_any_wgrad(dy, x, 3, 3, 1, 1, 1, False)
        r[f"werr_{mode}"] = ((dw - wr.grad).norm() / wr.grad.norm()).item()
    C_.conv_any_set_f32_split(True)
    r["fwd_miopen"] = t(lambda: F.conv2d(x, w, None, 1, 1))
    r["dgrad_miopen"] = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
    r["wgrad_miopen"] = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) and v > 1e-3 else v) for k, v in r.items()}), flush=True)
