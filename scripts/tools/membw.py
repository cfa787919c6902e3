"""Streaming bandwidth ceilings on this GPU (what the BN passes at 5.2-5.6 TB/s are measured
against): bf16 copy (1 read + 1 write stream), 2-input add (2 reads + 1 write), read-only sum."""
import json

import torch

n = 256 * 56 * 56 * 256  # one stage-1 ResNet-50 activation (205 M bf16 = 411 MB)
a = torch.randn(n, device="cuda").to(torch.bfloat16)
b = torch.randn(n, device="cuda").to(torch.bfloat16)
c = torch.empty_like(a)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


B = n * 2
for name, fn, nbytes in (("copy", lambda: c.copy_(a), 2 * B), ("add", lambda: torch.add(a, b, out=c), 3 * B),
                         ("sum", lambda: a.sum(dtype=torch.float32), B)):
    ms = t(fn)
    print(json.dumps({"op": name, "ms": round(ms, 4), "TB/s": round(nbytes / ms / 1e9, 2)}))
