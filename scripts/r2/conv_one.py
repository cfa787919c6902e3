"""Launch one native conv forward shape repeatedly (for rocprofv3 --pmc passes).
usage: conv_one.py Cin H Cout k s [bk stages occ [iters [tile]]]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.ops._ext import native  # noqa: E402


def main():
    a = [int(v) for v in sys.argv[1:]]
    Cin, H, Cout, k, s = a[:5]
    bk, st, occ = (a[5:8] + [0, 0, 0])[:3] if len(a) > 5 else (0, 0, 0)
    iters = a[8] if len(a) > 8 else 20
    tile = a[9] if len(a) > 9 else 0
    C_ = native()
    B = 256
    x = torch.randn(B, Cin, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).contiguous(
        memory_format=torch.channels_last)
    C_.conv_set_tile(tile)
    C_.conv_set_bk(bk)
    C_.conv_set_stages(st)
    C_.conv_set_occupancy(occ)
    for _ in range(iters):
        C_.conv2d_fwd(x, w, None, s, k // 2, False, True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
