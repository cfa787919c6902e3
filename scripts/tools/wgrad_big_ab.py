"""Per-shape time of the ResNet-50 b256 conv weight gradients on the 128 x 128 kernel
(conv_wgrad_k) and on the big-tile kernel (conv_wgrad_big_k), each alone on the GPU.

    python scripts/tools/wgrad_big_ab.py [--batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.ops._ext import native  # noqa: E402


def shapes(batch):
    m = models.resnet50(num_classes=1000)
    seen = []
    hooks = []
    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            def hook(mod, inp, out, seen=seen):
                key = (tuple(inp[0].shape), tuple(mod.weight.shape), mod.stride[0], mod.padding[0], tuple(out.shape))
                if key not in seen:
                    seen.append(key)
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(1, 3, 224, 224))
    for h in hooks:
        h.remove()
    out = []
    for (xs, ws, st, pad, ys) in seen:
        if xs[1] == 3:
            continue  # the stem has its own weight-gradient kernel
        out.append(((batch,) + xs[1:], ws, st, pad, (batch,) + ys[1:]))
    return out


def time_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    C = native()
    tot0 = tot1 = 0.0
    print(f"{'x':>22} {'w':>20} st  tile        small_ms  big_ms   TF/s(small) TF/s(big)")
    for xs, ws, st, pad, ys in shapes(a.batch):
        x = torch.randn(xs, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(ys, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        R = ws[2]
        npq = ys[0] * ys[2] * ys[3]
        flop = 2.0 * npq * ws[0] * ws[1] * R * R
        C.conv_wgrad_set_big(0)
        t0 = time_ms(lambda: C.conv2d_wgrad(dy, x, R, R, st, pad))
        C.conv_wgrad_set_big(1)
        code = C.conv_wgrad_big_choice(ws[1], ws[0], R, R, npq)
        t1 = time_ms(lambda: C.conv2d_wgrad(dy, x, R, R, st, pad)) if code else t0
        C.conv_wgrad_set_big(0)
        tile = f"{code >> 12}x{code & 0xfff}" if code else "-"
        tot0 += t0
        tot1 += t1
        print(f"{str(xs):>22} {str(ws):>20} {st}  {tile:10s} {t0:8.3f} {t1:8.3f}   {flop / t0 / 1e9:8.0f}  {flop / t1 / 1e9:8.0f}",
              flush=True)
    print(f"sum of unique shapes: small {tot0:.3f} ms, big where eligible {tot1:.3f} ms")


if __name__ == "__main__":
    main()
