"""Per-shape A/B of the big-tile conv kernel (csrc/conv_big.hip) against the 128x128 kernels
(csrc/conv.hip) on the ResNet-50 b256 shapes, in ONE process with interleaved rounds.

For every conv shape of the model (stem excluded): the forward with the BatchNorm-statistics
epilogue and, for stride-1 shapes, the input-gradient form with the BN-backward epilogue (the
flipped-weight conv2d_fwd call the backward makes).  Each variant is checked against an fp32
torch reference (outputs) and against the 128x128 kernel (statistics / partials summed over rows).
Prints one JSON line per (shape, kind, variant): median / min ms over the rounds and TFLOP/s.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.nn.functional as F


def shapes_resnet50():
    from torchbooster_amd.models import resnet50

    m = resnet50()
    seen = {}

    def mk(conv):
        def h(mod, inp, out):
            x = inp[0]
            key = (x.shape[1], x.shape[2], conv.out_channels, conv.kernel_size[0], conv.stride[0], conv.padding[0])
            seen[key] = seen.get(key, 0) + 1
        return h

    hooks = [mod.register_forward_hook(mk(mod)) for mod in m.modules() if isinstance(mod, torch.nn.Conv2d)]
    with torch.no_grad():
        m(torch.randn(1, 3, 224, 224))
    for h in hooks:
        h.remove()
    return seen


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--codes", default="")
    ap.add_argument("--kinds", default="fwd,dgrad")
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--only", default="", help="comma list of C:H:K:R:st shape filters")
    a = ap.parse_args()
    from torchbooster_amd.ops._ext import native

    C_ = native()
    enc = C_.conv_big_encode
    codes = [("old", 0)]
    if a.codes:
        for s in a.codes.split(";"):
            bm, bn, mf, st = (int(v) for v in s.split(","))
            codes.append((f"big{bm}x{bn}m{mf}s{st}", enc(bm, bn, mf, st)))
    else:
        codes += [("heur", 1)]
        for bm, bn, mf, st in [(128, 256, 16, 3), (128, 256, 32, 3), (128, 256, 16, 2), (64, 256, 16, 3),
                               (64, 256, 32, 3), (128, 128, 16, 4), (256, 256, 16, 2), (256, 128, 16, 3)]:
            codes.append((f"big{bm}x{bn}m{mf}s{st}", enc(bm, bn, mf, st)))
    dev = torch.device("cuda")
    B = a.batch
    torch.manual_seed(0)
    only = [tuple(int(v) for v in f.split(":")) for f in a.only.split(",") if f]
    for (C, H, K, R, st, pad), cnt in sorted(shapes_resnet50().items()):
        if C % 64 or K % 64:
            continue
        if only and not any((C, H, K, R, st) == o for o in only):
            continue
        P = (H + 2 * pad - R) // st + 1
        for kind in a.kinds.split(","):
            if kind == "dgrad" and st != 1:
                continue
            if kind == "fwd":
                x = cl(torch.randn(B, C, H, H, device=dev, dtype=torch.bfloat16))
                w = cl(torch.randn(K, C, R, R, device=dev, dtype=torch.bfloat16) * (1.0 / (C * R * R) ** 0.5))
                kw = dict(want_stats=True)
                cout, npq = K, B * P * P
                ref_fn = lambda: F.conv2d(x.float(), w.float(), stride=st, padding=pad)
            else:
                # input gradient of conv(C -> K): dY [B, K, P, P] conv'd with flipped weights -> dX [B, C, H, H]
                # plus the BN-backward partials of the BN in front of the conv (xb [B, C, H, H], ReLU bits)
                x = cl(torch.randn(B, K, P, P, device=dev, dtype=torch.bfloat16))
                w = cl(torch.randn(C, K, R, R, device=dev, dtype=torch.bfloat16) * (1.0 / (K * R * R) ** 0.5))
                xb = cl(torch.randn(B, C, H, H, device=dev, dtype=torch.bfloat16))
                mean = torch.randn(C, device=dev) * 0.1
                bits = torch.randint(0, 256, (B * H * H, C // 8), device=dev, dtype=torch.uint8)
                kw = dict(want_stats=False, bnb_mode=2, bnb_x=xb, bnb_mean=mean, bnb_bits=bits)
                cout, npq = C, B * H * H
                ref_fn = lambda: F.conv2d(x.float(), w.float(), stride=1, padding=pad)
            flop = 2.0 * npq * cout * (x.shape[1] * R * R)

            def run(code):
                C_.conv_set_big(code)
                return C_.conv2d_fwd(x, w, None, st if kind == "fwd" else 1, pad, False, kw.get("want_stats", False),
                                     **{k: v for k, v in kw.items() if k != "want_stats"})

            ok = {}
            if a.check:
                ref = ref_fn()
                base = None
                for name, code in codes:
                    outs = run(code)
                    torch.cuda.synchronize()
                    y, aux = outs[0], outs[1]
                    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                    colsum = aux.double().sum(0)
                    if base is None:
                        base = colsum
                    aerr = ((colsum - base).abs().max() / base.abs().max().clamp_min(1e-30)).item()
                    ok[name] = (err, aerr)
                del ref
            res = {name: [] for name, _ in codes}
            for _ in range(a.rounds):
                for name, code in codes:
                    run(code)
                    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                    s.record()
                    for _ in range(a.iters):
                        run(code)
                    e.record()
                    torch.cuda.synchronize()
                    res[name].append(s.elapsed_time(e) / a.iters)
            for name, _ in codes:
                ts = sorted(res[name])
                med = ts[len(ts) // 2]
                d = {"shape": [C, H, K, R, st, pad], "count": cnt, "kind": kind, "variant": name,
                     "ms_med": round(med, 4), "ms_min": round(ts[0], 4), "tflops": round(flop / med / 1e9, 1)}
                if name in ok:
                    d["rel_err"] = float(f"{ok[name][0]:.3g}")
                    d["aux_err"] = float(f"{ok[name][1]:.3g}")
                print(json.dumps(d), flush=True)
    C_.conv_set_big(0)


if __name__ == "__main__":
    main()
