"""Weight-gradient (TN) GEMMs dW[P][Q] = dyᵀ x over M rows: the 8-phase TN kernel (tile 16,
csrc/gemm8.hip) at several split counts vs the best of the 2-stage native tiles vs hipBLASLt.
ViT-B/16 b128 (M = 25216) and ResNet-50 b256 1x1-conv shapes.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.ops._ext import native  # noqa: E402

SHAPES = [  # (P = out, Q = in, M, label)
    (2304, 768, 25216, "vit_qkv_w"), (768, 768, 25216, "vit_proj_w"), (3072, 768, 25216, "vit_fc1_w"),
    (768, 3072, 25216, "vit_fc2_w"),
    (256, 64, 802816, "r50_l1_expand_w"), (64, 256, 802816, "r50_l1_reduce_w"), (512, 128, 200704, "r50_l2_expand_w"),
    (128, 512, 200704, "r50_l2_reduce_w"), (1024, 256, 50176, "r50_l3_expand_w"), (256, 1024, 50176, "r50_l3_reduce_w"),
    (2048, 512, 12544, "r50_l4_expand_w"), (512, 2048, 12544, "r50_l4_reduce_w"),
]


def timeit(fn, reps=10):
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
    for P, Q, M, lab in SHAPES:
        dy = (torch.rand(M, P, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(M, Q, device="cuda") * 2 - 1).to(torch.bfloat16)
        fl = 2.0 * P * Q * M
        out = {"shape": lab, "P": P, "Q": Q, "M": M}
        ref = dy[:4096].float().t() @ x[:4096].float()
        y = C.gemm(dy[:4096], x[:4096], True, tx=True, tile=16, splits=4)[0]
        out["rel_err_t16"] = round(((y.float() - ref).norm() / ref.norm()).item(), 6)
        best = {}
        for s in (1, 2, 4, 8, 16, 32):
            best[f"t16s{s}"] = timeit(lambda: C.gemm(dy, x, True, tx=True, tile=16, splits=s))
        for t in (0, 1, 3, 5):
            for s in (1, 4, 8, 16):
                try:
                    best[f"t{t}s{s}"] = timeit(lambda: C.gemm(dy, x, True, tx=True, tile=t, splits=s))
                except RuntimeError:
                    pass
        best["blas"] = timeit(lambda: dy.t() @ x)
        k16 = min((k for k in best if k.startswith("t16")), key=best.get)
        knat = min((k for k in best if k.startswith("t") and not k.startswith("t16")), key=best.get)
        out.update({"t16_best": k16, "t16_ms": round(best[k16], 4), "t16_tf": round(fl / best[k16] / 1e9, 1),
                    "old_best": knat, "old_ms": round(best[knat], 4), "old_tf": round(fl / best[knat] / 1e9, 1),
                    "blas_ms": round(best["blas"], 4), "blas_tf": round(fl / best["blas"] / 1e9, 1),
                    "all": {k: round(v, 4) for k, v in best.items()}})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
