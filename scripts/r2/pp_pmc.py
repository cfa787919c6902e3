"""4096^3 GEMMs for a PMC pass: gemm.hip tile 0, ping-pong tile 16, torch (hipBLASLt)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from torchbooster_amd.ops._ext import native
C = native()
n = int(os.environ.get("N", "4096"))
x = torch.randn(n, n, device="cuda").to(torch.bfloat16)
w = torch.randn(n, n, device="cuda").to(torch.bfloat16)
for tile in [int(t) for t in os.environ.get("TILES", "0,16").split(",")]:
    for _ in range(10):
        C.gemm(x, w, False, tile=tile)
for _ in range(10):
    x @ w.t()
torch.cuda.synchronize()
