"""Cost of a cross-stream fork (event record on the compute stream + wait on a side stream)
between back-to-back kernels: the per-conv wgrad side-stream fork of ops/streams.py."""
import json
import time

import torch


def run(n, fork, side, x, work):
    main = torch.cuda.current_stream()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        x.mul_(1.0000001)
        if fork:
            side.wait_stream(main)
            if work:
                with torch.cuda.stream(side):
                    torch.cuda.current_stream()  # no kernel
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    torch.cuda.set_device(0)
    side = torch.cuda.Stream()
    out = {}
    for numel in (1 << 16, 1 << 24):
        x = torch.ones(numel, device="cuda")
        for fork in (False, True):
            run(50, fork, side, x, False)
            t = min(run(400, fork, side, x, False) for _ in range(3))
            out[f"n{numel}_fork{int(fork)}_us_per_kernel"] = round(t, 2)
    # host cost of a launch + fork
    x = torch.ones(1 << 16, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        x.mul_(1.0000001)
    out["host_us_per_launch"] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        side.wait_stream(torch.cuda.current_stream())
    out["host_us_per_fork"] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
