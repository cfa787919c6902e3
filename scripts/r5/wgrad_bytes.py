"""Per-shape weight-gradient traffic: every ResNet-50 b256 weight gradient (the shipped wgrad route
rows) run alone, 3x each, so a rocprofv3 FETCH_SIZE / WRITE_SIZE pass can be compared with the
operand minimum |X| + |dY| (bf16) + the split-K partials (f32, written once and read once).

python scripts/r5/wgrad_bytes.py [--list]   (prints one line per shape: key, minimum MB)"""
import json
import sys

import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchbooster_amd.ops import _ext  # noqa: E402

ROUTES = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      "torchbooster_amd", "ops", "conv_routes_gfx950.json")


def shapes():
    out = []
    for key, name in json.load(open(ROUTES))["routes"]:
        if key[0] == "wgrad" and isinstance(key[1], list) and key[1][0] == 256 and len(key) == 5:
            x, w, stride, pad = key[1], key[2], key[3], key[4]
            out.append((tuple(x), tuple(w), stride, pad))
    return out


def main():
    nat = _ext.native()
    for x, w, stride, pad in shapes():
        N, C, H, W = x
        K, _, R, S = w
        P = (H + 2 * pad - R) // stride + 1
        Q = (W + 2 * pad - S) // stride + 1
        mb = (N * H * W * C + N * P * Q * K) * 2 / 2**20
        ws = nat.conv_wgrad_workspace_floats(N, H, W, C, K, R, S, P, Q, stride, pad) if hasattr(
            nat, "conv_wgrad_workspace_floats") else -1
        print(f"shape x={x} w={w} s={stride} p={pad} min_operand_MB={mb:.1f} partial_floats={ws}", flush=True)
        if "--list" in sys.argv:
            continue
        xt = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, K, P, Q, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        for _ in range(3):
            nat.conv2d_wgrad(dy, xt, R, S, stride, pad)
        torch.cuda.synchronize()
        del xt, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
