"""Workload for the gemm8 PMC passes: hipBLASLt, gemm8 (staggered / not) and tile 0 on 4096^3 and a
ViT fc1 shape, 5 dispatches each, random operands."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.ops._ext import native  # noqa: E402

C = native()
for P, Q, K in ((4096, 4096, 4096), (25216, 3072, 768)):
    x = (torch.rand(P, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(Q, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    for _ in range(5):
        x @ w.t()
    for st in (1, 0):
        C.gemm8_set_stagger(st)
        for _ in range(5):
            C.gemm(x, w, False, tile=16)
    for _ in range(5):
        C.gemm(x, w, False, tile=0)
    torch.cuda.synchronize()
