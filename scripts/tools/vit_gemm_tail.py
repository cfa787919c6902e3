"""ViT GEMM shapes: the 8-phase kernel over the whole grid (tile 16) vs whole rounds + 128x128 tail
(tiles 17 / 18) vs hipBLASLt (ATen); ms, TF/s and max |diff| of 17/18 against tile 16."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd.ops._ext import native  # noqa: E402

C = native()


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
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


shapes = []
for T in (25216, 50432):
    shapes += [("proj_fwd", "nt", T, 768, 768), ("fc2_fwd", "nt", T, 768, 3072), ("qkv_dgrad", "nn", T, 768, 2304),
               ("fc1_dgrad", "nn", T, 768, 3072), ("proj_dgrad", "nn", T, 768, 768), ("qkv_fwd", "nt", T, 2304, 768),
               ("fc1_fwd", "nt", T, 3072, 768)]
shapes += [("s_proj_fwd", "nt", 25216, 384, 384), ("s_fc2_fwd", "nt", 25216, 384, 1536)]
for name, kind, T, Q, K in shapes:
    x = r(T, K)
    if kind == "nt":
        w = r(Q, K)
        b = r(Q)
        f = {f"t{tl}": (lambda tl=tl: C.gemm(x, w, False, bias=b, epi=1, tile=tl, splits=1)[0]) for tl in (16, 17, 18)}
        f["blas"] = lambda: torch.nn.functional.linear(x, w, b)
    else:
        w = r(K, Q)
        f = {f"t{tl}": (lambda tl=tl: C.gemm(x, w, True, tile=tl, splits=1)[0]) for tl in (16, 17, 18)}
        f["blas"] = lambda: x @ w
    fl = 2 * T * Q * K / 1e12
    row = {"shape": name, "P": T, "Q": Q, "K": K}
    ref = f["t16"]().float()
    for k in ("t17", "t18"):
        row[k + "_maxdiff"] = float((f[k]().float() - ref).abs().max())
    for k, fn in f.items():
        ms = t(fn)
        row[k] = round(ms, 4)
        row[k + "_tf"] = round(fl / ms * 1e3)
    print(json.dumps(row), flush=True)
