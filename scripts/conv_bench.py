"""Per-shape conv timing for ResNet-50 b256 bf16 NHWC: MIOpen (ATen) vs GEMM (hipBLASLt) vs native.

Prints one JSON line per shape with fwd / dgrad / wgrad ms and TFLOP/s.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def shapes_resnet50(B):
    from torchbooster_amd.models import resnet50

    m = resnet50()
    seen = {}
    hooks = []

    def mk(conv):
        def h(mod, inp, out):
            x = inp[0]
            key = (x.shape[1], x.shape[2], x.shape[3], conv.out_channels, conv.kernel_size[0], conv.stride[0],
                   conv.padding[0])
            seen[key] = seen.get(key, 0) + 1
        return h

    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            hooks.append(mod.register_forward_hook(mk(mod)))
    with torch.no_grad():
        m(torch.randn(1, 3, 224, 224))
    return seen


def timeit(fn, iters=10, warm=3):
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
    ap.add_argument("--native", action="store_true")
    ap.add_argument("--native-only", action="store_true")
    ap.add_argument("--dgrad", action="store_true", help="also time native dgrad (stride 1)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    B = a.batch
    dev = "cuda"
    tot = {"miopen": 0.0, "gemm": 0.0, "native": 0.0}
    for (Cin, H, W, Cout, k, s, p), cnt in sorted(shapes_resnet50(B).items()):
        x = torch.randn(B, Cin, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Cout, Cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, w, None, s, p)
        dy = torch.randn_like(y)
        Ho, Wo = y.shape[2], y.shape[3]
        flop = 2.0 * B * Ho * Wo * Cout * Cin * k * k
        r = {"Cin": Cin, "H": H, "Cout": Cout, "k": k, "s": s, "count": cnt}
        f = lambda: F.conv2d(x, w, None, s, p)
        bd = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                          [True, False, False])
        bw = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                          [False, True, False])
        if not a.native_only:
            r["miopen_ms"] = [round(timeit(f), 4), round(timeit(bd), 4), round(timeit(bw), 4)]
            r["miopen_tflops"] = [round(flop / (t * 1e9), 1) for t in r["miopen_ms"]]
            tot["miopen"] += cnt * sum(r["miopen_ms"])
        if a.native_only:
            pass
        elif k == 1:
            xs = x if s == 1 else x[:, :, ::s, ::s]
            x2 = xs.permute(0, 2, 3, 1).reshape(-1, Cin)
            w2 = w.reshape(Cout, Cin)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, Cout)
            g = [timeit(lambda: torch.mm(x2, w2.t())), timeit(lambda: torch.mm(dy2, w2)),
                 timeit(lambda: torch.mm(dy2.t(), x2))]
            if s != 1:
                g[0] += timeit(lambda: xs.contiguous(memory_format=torch.channels_last))
            r["gemm_ms"] = [round(t, 4) for t in g]
            r["gemm_tflops"] = [round(flop / (t * 1e9), 1) for t in g]
            tot["gemm"] += cnt * sum(min(a_, b_) for a_, b_ in zip(g, r["miopen_ms"]))
        else:
            tot["gemm"] += cnt * sum(r["miopen_ms"])
        if a.native or a.native_only:
            from torchbooster_amd.ops import conv as nconv

            try:
                nf = lambda: nconv.conv2d_forward(x, w, s, p)
                r["native_ms"] = [round(timeit(nf), 4)]
                r["native_tflops"] = [round(flop / (r["native_ms"][0] * 1e9), 1)]
                ref = F.conv2d(x.float(), w.float(), None, s, p)
                r["native_relerr"] = round(((nf().float() - ref).abs().max() / ref.abs().max()).item(), 5)
                tot["native"] += cnt * r["native_ms"][0]
                from torchbooster_amd.ops._ext import native as _nat
                if a.dgrad and s == 1:
                    wt = _nat().conv_flip_weight(w)
                    nd = lambda: _nat().conv2d_fwd(dy, wt, None, 1, k - 1 - p, False, False)[0]
                    r["native_dgrad_ms"] = round(timeit(nd), 4)
                if a.dgrad:
                    nw = lambda: _nat().conv2d_wgrad(dy, x, k, k, s, p)
                    r["native_wgrad_ms"] = round(timeit(nw), 4)
                    r["native_wgrad_tflops"] = round(flop / (r["native_wgrad_ms"] * 1e9), 1)
                    wref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [s, s], [p, p],
                                                               [1, 1], False, [0, 0], 1, [False, True, False])[1]
                    r["native_wgrad_relerr"] = round(((nw().float() - wref).abs().max() / wref.abs().max()).item(), 5)
                    tot["native_wgrad"] = tot.get("native_wgrad", 0.0) + cnt * r["native_wgrad_ms"]
            except Exception as e:  # shape not supported natively
                r["native_err"] = str(e)[:80]
        print(json.dumps(r), flush=True)
    print(json.dumps({"total_ms_per_step": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
