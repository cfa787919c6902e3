"""conv_any (csrc/conv_any.hip) vs MIOpen (ATen) per direction on the reference's small-channel /
fp32 shapes.  One JSON line per (shape, dtype)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
from torchbooster_amd.ops._ext import native

SHAPES = [  # N, C, H, K, R, stride, pad, up, reflect, label
    (256, 1, 28, 6, 5, 1, 0, 1, False, "lenet_c1"), (256, 6, 12, 16, 5, 1, 0, 1, False, "lenet_c2"),
    (8, 3, 256, 32, 9, 1, 4, 1, True, "style_in"), (8, 32, 256, 64, 3, 2, 1, 1, True, "style_down1"),
    (8, 128, 64, 64, 3, 1, 1, 2, True, "style_up1"), (8, 32, 256, 3, 9, 1, 4, 1, True, "style_out"),
    (32, 64, 128, 3, 9, 1, 4, 1, True, "adain_out"),
    (1, 64, 512, 64, 3, 1, 1, 1, False, "vgg_512_c64"), (1, 256, 128, 256, 3, 1, 1, 1, False, "vgg_128_c256"),
    (128, 3, 128, 64, 4, 2, 1, 1, False, "dcgan_d_in"),  # its dgrad / wgrad = the G output ConvT fwd / wgrad
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    C_ = native()
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    dts = (torch.bfloat16,) if os.environ.get("BF16_ONLY") else (torch.float32, torch.bfloat16)
    for N, C, H, K, R, st, pad, up, refl, lab in SHAPES:
        if only and lab not in only:
            continue
        for dt in dts:
            x = torch.randn(N, C, H, H, device="cuda", dtype=dt).contiguous(memory_format=torch.channels_last)
            w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).to(dt)
            mode = "reflect" if refl else "constant"

            def ref_fwd():
                xx = F.interpolate(x, scale_factor=up, mode="nearest") if up > 1 else x
                xx = F.pad(xx, (pad,) * 4, mode=mode) if pad else xx
                return F.conv2d(xx, w, None, st)

            y = ref_fwd()
            dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
            xp = (F.pad(F.interpolate(x, scale_factor=up, mode="nearest") if up > 1 else x, (pad,) * 4, mode=mode)
                  if pad else x).contiguous(memory_format=torch.channels_last)
            r = {"shape": lab, "dtype": str(dt).split(".")[1]}
            r["fwd_any"] = timeit(lambda: C_.conv_any_fwd(x, w, None, st, pad, up, refl))
            r["fwd_miopen"] = timeit(ref_fwd)
            r["dgrad_any"] = timeit(lambda: C_.conv_any_dgrad(dy, w, H, H, st, pad, up, refl))
            r["dgrad_miopen_padded"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, xp, w, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
            r["wgrad_any"] = timeit(lambda: C_.conv_any_wgrad(dy, x, R, R, st, pad, up, refl))
            r["wgrad_miopen_padded"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, xp, w, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
