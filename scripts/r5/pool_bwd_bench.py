"""ResNet stem backward at b256: max-pool gather + BN backward (unfused) against the fused
bn_backward_pool (pool_gather.h inside the BN partial / apply passes); interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from torchbooster_amd.ops._ext import native

C_ = native()
N, C, H = int(os.environ.get("B", "256")), 64, 112
P = 56
dev = "cuda"
x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
rows = x.permute(0, 2, 3, 1).reshape(-1, C)
w = torch.rand(C, device=dev) + 0.5
b = torch.randn(C, device=dev) * 0.2
mean, invstd, scale, shift = C_.bn_stats(rows, None, w, b, None, None, True, 0.1, 1e-5, None)
y, idx = C_.bn_act_maxpool(x, scale, shift, 1, 0.0, 3, 2, 1)
dy = torch.randn_like(y)


def unfused():
    dz = C_.maxpool_backward(dy, idx, H, H, 3, 2, 1)
    dzr = dz.permute(0, 2, 3, 1).reshape(-1, C)
    return C_.bn_backward(dzr, rows, rows, None, w, mean, invstd, scale, shift, True, 1, 0.0, False, None, None)[:3]


def fused():
    return C_.bn_backward_pool(dy, idx, rows, N, H, H, 3, 2, 1, w, mean, invstd, scale, shift, True, 1, 0.0)


a, f = unfused(), fused()
torch.cuda.synchronize()
for name, u, v in zip(("dx", "dgamma", "dbeta"), a, f):
    print(name, "rel diff", ((u.float() - v.float()).norm() / u.float().norm()).item())
res = {"unfused": [], "fused": []}
for _ in range(5):
    for name, fn in (("unfused", unfused), ("fused", fused)):
        fn()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name].append(s.elapsed_time(e) / 10)
for k, v in res.items():
    v.sort()
    print(k, "ms med", round(v[2], 4), "min", round(v[0], 4))
