"""ViT-B/16 b128 (25216 tokens) N = 768 products: the 8-phase kernel whole vs tail split-K
(S = 2, 3) vs hipBLASLt (ATen), ms and TF/s per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd.ops._ext import native  # noqa: E402

C = native()
T = 25216


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def r(*s):
    return (torch.randn(*s, device="cuda") * 0.05).to(torch.bfloat16)


for name, kind, Q, K in (("proj_fwd", "nt", 768, 768), ("fc2_fwd", "nt", 768, 3072), ("qkv_dgrad", "nn", 768, 2304),
                         ("fc1_dgrad", "nn", 768, 3072), ("proj_dgrad", "nn", 768, 768), ("qkv_fwd", "nt", 2304, 768),
                         ("fc1_fwd", "nt", 3072, 768)):
    x = r(T, K)
    if kind == "nt":
        w = r(Q, K)
        b = r(Q)
        f = {f"s{s}": (lambda s=s: C.gemm(x, w, False, bias=b, epi=1, tile=16, splits=s)) for s in (1, 2, 3)}
        f["blas"] = lambda: torch.nn.functional.linear(x, w, b)
    else:
        w = r(K, Q)
        f = {f"s{s}": (lambda s=s: C.gemm(x, w, True, tile=16, splits=s)) for s in (1, 2, 3)}
        f["blas"] = lambda: x @ w
    fl = 2 * T * Q * K / 1e12
    row = {"shape": name, "P": T, "Q": Q, "K": K}
    for k, fn in f.items():
        ms = t(fn)
        row[k] = round(ms, 4)
        row[k + "_tf"] = round(fl / ms * 1e3)
    print(json.dumps(row), flush=True)
