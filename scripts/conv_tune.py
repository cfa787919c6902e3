"""Sweep the native conv pipeline depth (LDS stages) per ResNet-50 shape.

For every (shape, stages) prints fwd / dgrad ms and TFLOP/s plus a numerics
check against an fp32 reference; ends with the best stage count per shape.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from conv_bench import shapes_resnet50, timeit  # noqa: E402
from torchbooster_amd.ops._ext import native  # noqa: E402


def main():
    B = int(os.environ.get("BATCH", "256"))
    C_ = native()
    best = {}
    for (Cin, H, W, Cout, k, s, p), cnt in sorted(shapes_resnet50(B).items()):
        if Cin % 64:
            continue
        x = torch.randn(B, Cin, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Cout, Cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        ref = F.conv2d(x.float(), w.float(), None, s, p)
        dy = torch.randn(ref.shape, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = C_.conv_flip_weight(w)
        flop = 2.0 * ref.numel() * Cin * k * k
        row = {"shape": [Cin, H, Cout, k, s], "count": cnt}
        for st, occ in ((1, 2), (1, 3), (1, 4), (2, 2)):
            C_.conv_set_stages(st)
            C_.conv_set_occupancy(occ)
            st = f"{st}o{occ}"
            y = C_.conv2d_fwd(x, w, None, s, p, False, False)[0]
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            tf = timeit(lambda: C_.conv2d_fwd(x, w, None, s, p, False, False))
            row[f"fwd_s{st}"] = [round(tf, 4), round(flop / tf / 1e9, 1), round(err, 4)]
            if s == 1:
                td = timeit(lambda: C_.conv2d_fwd(dy, wt, None, 1, k - 1 - p, False, False))
                row[f"dgrad_s{st}"] = [round(td, 4), round(flop / td / 1e9, 1)]
        C_.conv_set_stages(0)
        C_.conv_set_occupancy(0)
        wref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [s, s], [p, p], [1, 1],
                                                   False, [0, 0], 1, [False, True, False])[1]
        for st in ("1o2", "1o3", "1o4"):  # (the weight gradient is single-stage only)
            C_.conv_wgrad_set_occupancy(int(st[2]))
            dw = C_.conv2d_wgrad(dy, x, k, k, s, p)
            err = ((dw.float() - wref).abs().max() / wref.abs().max()).item()
            tw = timeit(lambda: C_.conv2d_wgrad(dy, x, k, k, s, p))
            row[f"wgrad_s{st}"] = [round(tw, 4), round(flop / tw / 1e9, 1), round(err, 4)]
        C_.conv_wgrad_set_occupancy(0)
        row["best_wgrad"] = min(("1o2", "1o3", "1o4"), key=lambda st: row[f"wgrad_s{st}"][0])
        keys = ["1o2", "1o3", "1o4", "2o2"]
        row["best_fwd"] = min(keys, key=lambda st: row[f"fwd_s{st}"][0])
        if s == 1:
            row["best_dgrad"] = min(keys, key=lambda st: row[f"dgrad_s{st}"][0])
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
