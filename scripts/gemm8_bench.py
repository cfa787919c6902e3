"""The 8-phase 256x256 NT kernel (csrc/gemm8.hip, tile 16) vs hipBLASLt (torch) vs the
2-stage / split-half 256x256 tiles of csrc/gemm.hip on the framework's NT shapes.
Random uniform operands (cdna_hip_programming.md rule 25).  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchbooster_amd.ops._ext import native  # noqa: E402

SHAPES = [  # (P, Q, K, label)
    (4096, 4096, 4096, "square4k"), (8192, 8192, 8192, "square8k"),
    (25216, 2304, 768, "vit_qkv"), (25216, 768, 768, "vit_proj"), (25216, 3072, 768, "vit_fc1"),
    (25216, 768, 3072, "vit_fc2"),
    (802816, 256, 64, "r50_l1_expand"), (802816, 64, 256, "r50_l1_reduce"), (200704, 512, 128, "r50_l2_expand"),
    (200704, 128, 512, "r50_l2_reduce"), (50176, 1024, 256, "r50_l3_expand"), (50176, 256, 1024, "r50_l3_reduce"),
    (12544, 2048, 512, "r50_l4_expand"), (12544, 512, 2048, "r50_l4_reduce"),
    (1000, 520, 192, "tail_odd"),
]


def timeit(fn, reps=20):
    for _ in range(3):
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
    C = native()
    torch.manual_seed(0)
    for P, Q, K, lab in SHAPES:
        x = (torch.rand(P, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(Q, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        fl = 2.0 * P * Q * K
        out = {"shape": lab, "P": P, "Q": Q, "K": K}
        C.gemm8_set_stagger(1)
        y8 = C.gemm(x, w, False, tile=16)[0]
        ref = x[:2048].float() @ w.float().t()
        err = ((y8[:2048].float() - ref).norm() / ref.norm()).item()
        out["rel_err_t16"] = err
        C.gemm8_set_stagger(0)
        y8 = C.gemm(x, w, False, tile=16)[0]
        out["rel_err_t16ns"] = ((y8[:2048].float() - ref).norm() / ref.norm()).item()
        def t16(stagger):
            C.gemm8_set_stagger(stagger)
            return C.gemm(x, w, False, tile=16)

        for name, fn in (("blas", lambda: x @ w.t()), ("t16", lambda: t16(1)), ("t16ns", lambda: t16(0)),
                         ("t0", lambda: C.gemm(x, w, False, tile=0)), ("t10", lambda: C.gemm(x, w, False, tile=10)),
                         ("t1", lambda: C.gemm(x, w, False, tile=1))):
            ms = timeit(fn)
            out[name + "_ms"] = round(ms, 4)
            out[name + "_tf"] = round(fl / ms / 1e9, 1)
        print(json.dumps(out), flush=True)
        del x, w, y8


if __name__ == "__main__":
    main()
