"""Forward / stride-1 dgrad conv kernel variants per ResNet-50 shape (b256, bf16, NHWC):
the default 64-deep single-stage kernel vs 32-deep k-tiles in 2-4 stage rings.
One JSON line per shape: ms, TF/s and max-rel error vs fp32 per variant."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import shapes_resnet50, timeit  # noqa: E402
from torchbooster_amd.ops._ext import native  # noqa: E402

# (name, k-tile depth, stages, occupancy, tile: 0 auto / 1 = 128ch x 256px / 2 = 256ch x 128px)
# bk >= 100: 64-deep single stage scheduled with __builtin_amdgcn_iglp_opt(bk - 100)
VARIANTS = [("64s1", 64, 1, 0, 0), ("prio1", 64, 1, 0, 0), ("prio3", 64, 1, 0, 0)]

# wgrad: (name, stages knob (>= 100: iglp_opt(knob - 100)), occupancy)
WG_VARIANTS = []


def main():
    B = int(os.environ.get("BATCH", "256"))
    C_ = native()
    tot = {v[0]: 0.0 for v in VARIANTS}
    for (Cin, H, W, Cout, k, s, p), cnt in sorted(shapes_resnet50(B).items()):
        if Cin % 64:
            continue
        torch.manual_seed(0)
        x = torch.randn(B, Cin, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Cout, Cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        ref = F.conv2d(x.float(), w.float(), None, s, p)
        flop = 2.0 * ref.numel() * Cin * k * k
        row = {"shape": [Cin, H, Cout, k, s], "count": cnt}
        for name, bk, st, occ, tile in VARIANTS:
            if hasattr(C_, "conv_set_prio"):  # study knob (a3fe7df-era builds / the setprio study)
                C_.conv_set_prio(int(name[4:]) if name.startswith("prio") else 0)
            y, st_ = C_.conv2d_fwd(x, w, None, s, p, False, True)[:2]
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            ssum = st_[:, 0].sum(0)
            serr = ((ssum - y.float().sum((0, 2, 3))).abs().max() / y.float().abs().sum((0, 2, 3)).max()).item()
            t = timeit(lambda: C_.conv2d_fwd(x, w, None, s, p, False, True), iters=20)
            row[name] = [round(t, 4), round(flop / t / 1e9, 1), round(err, 4), round(serr, 6)]
            tot[name] += t * cnt
        for name, *_ in VARIANTS:  # totals count the default where a variant does not apply
            if name not in row:
                tot[name] += row["64s1"][0] * cnt
        if hasattr(C_, "conv_set_prio"):
            C_.conv_set_prio(0)
        row["best"] = min((v[0] for v in VARIANTS if v[0] in row), key=lambda n: row[n][0])
        if os.environ.get("WGRAD", "1") == "1":
            dy = torch.randn(ref.shape, device="cuda", dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            wref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [s, s], [p, p],
                                                       [1, 1], False, [0, 0], 1, [False, True, False])[1]
            for name, stg, occ in WG_VARIANTS:
                C_.conv_wgrad_set_stages(stg)
                C_.conv_wgrad_set_occupancy(occ)
                dw = C_.conv2d_wgrad(dy, x, k, k, s, p)
                err = ((dw.float() - wref).abs().max() / wref.abs().max()).item()
                t = timeit(lambda: C_.conv2d_wgrad(dy, x, k, k, s, p), iters=20)
                row[name] = [round(t, 4), round(flop / t / 1e9, 1), round(err, 4)]
                tot[name] = tot.get(name, 0.0) + t * cnt
            C_.conv_wgrad_set_stages(0)
            C_.conv_wgrad_set_occupancy(0)
            row["best_w"] = min((v[0] for v in WG_VARIANTS), key=lambda n: row[n][0])
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
