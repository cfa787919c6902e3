"""BatchNorm(+ReLU, +residual) kernel bandwidth on ResNet-50 b256 activation shapes.

For each (M = N*H*W, C, residual) prints the forward (statistics from the conv
epilogue -> apply) and backward (partial -> finalize -> apply) time and the
achieved HBM bandwidth counting the minimum bytes each direction must move.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from torchbooster_amd.ops._ext import native

SHAPES = [  # (H, C, residual, count) for ResNet-50 at 224 px
    (112, 64, False, 1), (56, 64, False, 6), (56, 256, True, 3), (56, 256, False, 1), (56, 128, False, 1),
    (28, 128, False, 7), (28, 512, True, 4), (28, 512, False, 1), (28, 256, False, 1), (14, 256, False, 11),
    (14, 1024, True, 6), (14, 1024, False, 1), (14, 512, False, 1), (7, 512, False, 5), (7, 2048, True, 3),
    (7, 2048, False, 1),
]


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    C_ = native()
    dev = "cuda"
    tot_f = tot_b = 0.0
    for H, C, res, cnt in SHAPES:
        M = a.batch * H * H
        x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
        r = torch.randn(M, C, device=dev, dtype=torch.bfloat16) if res else None
        g = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        # conv-epilogue style statistics: one tile of raw sums
        xf = x.float()
        stats = torch.stack([xf.sum(0), (xf * xf).sum(0)]).unsqueeze(0).contiguous()
        del xf
        fwd = lambda: C_.bn_forward_from_stats(x, stats, g, b, rm, rv, 0.1, 1e-5, r, 1, 0.0)
        y, mean, invstd, scale, shift, _ = fwd()
        dy = torch.randn_like(x)
        bwd = lambda: C_.bn_backward(dy, y, x, None, g, mean, invstd, scale, shift, True, 1, 0.0, res)
        tf, tb = timeit(fwd), timeit(bwd)
        e = M * C * 2
        bf = e * (3 if res else 2)            # read x (+res), write y
        bb = e * (2 + 3 + (1 if res else 0))  # partial: dy, y ; apply: dy, x, write dx (+ dres)
        out = {"M": M, "C": C, "res": res, "count": cnt, "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
               "fwd_GBs": round(bf / tf / 1e6, 1), "bwd_GBs": round(bb / tb / 1e6, 1)}
        tot_f += cnt * tf
        tot_b += cnt * tb
        print(json.dumps(out), flush=True)
    print(json.dumps({"total_ms_per_step": {"fwd": round(tot_f, 3), "bwd": round(tot_b, 3)}}), flush=True)


if __name__ == "__main__":
    main()
