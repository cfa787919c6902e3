"""1x1 stride-1 ResNet-50 (b256) convs: native implicit-GEMM conv kernel vs the native GEMM
engine (tuned tiles incl. the 8-phase 256x256) vs hipBLASLt, forward / dgrad / wgrad."""
import json, sys
import torch
import torch.nn.functional as F
from torchbooster_amd.ops._ext import native
from torchbooster_amd.ops import gemm as G

SH = [(64, 64, 56), (64, 256, 56), (256, 64, 56), (256, 128, 56), (128, 512, 28), (512, 128, 28),
      (512, 256, 28), (256, 1024, 14), (1024, 256, 14), (1024, 512, 14), (512, 2048, 7), (2048, 512, 7)]
N = 256


def t(fn, reps=20):
    fn(); fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps):
        fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps


for C, K, H in SH:
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 1, 1, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
    w2 = w.view(K, C)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, K)
    wt = native().conv_flip_weight(w)
    r = {"C": C, "K": K, "H": H, "px": x2.shape[0]}
    r["conv_fwd"] = t(lambda: native().conv2d_fwd(x, w, None, 1, 0, False, False))
    r["conv_fwd_stats"] = t(lambda: native().conv2d_fwd(x, w, None, 1, 0, True, False))
    r["gemm_fwd"] = t(lambda: G.mm_nt(x2, w2, blas=False))
    r["blas_fwd"] = t(lambda: F.linear(x2, w2))
    r["conv_dgrad"] = t(lambda: native().conv2d_fwd(dy, wt, None, 1, 0, False, False))
    r["gemm_dgrad"] = t(lambda: G.mm_nn(dy2, w2))
    r["blas_dgrad"] = t(lambda: dy2 @ w2)
    r["conv_wgrad"] = t(lambda: native().conv2d_wgrad(dy, x, 1, 1, 1, 0))
    r["gemm_wgrad"] = t(lambda: G.mm_tn(dy2, x2))
    r["blas_wgrad"] = t(lambda: dy2.t() @ x2)
    mb = (x.numel() + dy.numel()) * 2 / 1e6
    r["min_fwd_ms_at_5TBs"] = mb / 5e6 * 1e3
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
