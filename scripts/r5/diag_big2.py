"""Old (128x128) vs big-tile conv outputs/stats on small-NPQ shapes (bitwise: same k order)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from torchbooster_amd.ops._ext import native

C_ = native()
torch.manual_seed(0)
enc = C_.conv_big_encode
for (N, C, H, K, R, st, pad) in [(4, 2048, 2, 512, 1, 1, 0), (4, 512, 2, 512, 3, 1, 1), (4, 512, 2, 2048, 1, 1, 0),
                                 (4, 512, 4, 512, 3, 2, 1), (4, 1024, 4, 2048, 1, 2, 0), (4, 1024, 4, 256, 1, 1, 0),
                                 (4, 256, 4, 256, 3, 1, 1), (16, 512, 2, 512, 3, 1, 1), (1, 512, 7, 512, 3, 1, 1),
                                 (4, 128, 8, 128, 3, 1, 1)]:
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    res = []
    C_.conv_set_big(0)
    y0, s0 = C_.conv2d_fwd(x, w, None, st, pad, False, True)
    for code in [1, enc(128, 128, 16, 4), enc(128, 256, 16, 3), enc(256, 128, 16, 3)]:
        C_.conv_set_big(code)
        y1, s1 = C_.conv2d_fwd(x, w, None, st, pad, False, True)
        torch.cuda.synchronize()
        dy = (y1.float() - y0.float()).abs().max().item()
        ds = ((s1.double().sum(0) - s0.double().sum(0)).abs().max() / s0.double().sum(0).abs().max()).item()
        res.append(f"{code}: y {dy:.3g} st {ds:.3g} rows {s1.shape[0]}/{s0.shape[0]} nan {bool(torch.isnan(y1.float()).any())}")
    print((N, C, H, K, R, st, pad), "NPQ", y0.shape[0] * y0.shape[2] * y0.shape[3], " | ".join(res), flush=True)
C_.conv_set_big(0)
