"""ViT-B/16 fc2 input gradient + fc1 GELU backward + fc1 bias gradient, b128 (25216 tokens):
fused (one 8-phase NN GEMM with the GELU-backward epilogue) vs unfused (tuned NN GEMM + the
gelu_bwd_colsum pass) vs hipBLASLt + the same pass.  Also the plain NN (dgrad) shapes of ViT
on the 8-phase NN kernel vs the old tiles vs hipBLASLt."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd.ops._ext import native  # noqa: E402


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
    P, K, Q = 25216, 768, 3072
    dy = (torch.rand(P, K, device="cuda") - 0.5).to(torch.bfloat16)
    w = (torch.rand(K, Q, device="cuda") - 0.5).to(torch.bfloat16)
    z = (torch.rand(P, Q, device="cuda") * 4 - 2).to(torch.bfloat16)
    r = {"fused_ms": timeit(lambda: C.gemm_nn_gelu_bwd(dy, w, z))}
    for t in (0, 16):
        r[f"unfused_t{t}_ms"] = timeit(lambda: C.gelu_bwd_colsum(C.gemm(dy, w, True, tile=t)[0], z))
        r[f"nn_t{t}_ms"] = timeit(lambda: C.gemm(dy, w, True, tile=t))
    r["unfused_blas_ms"] = timeit(lambda: C.gelu_bwd_colsum(dy @ w, z))
    r["gelu_pass_ms"] = timeit(lambda: C.gelu_bwd_colsum(z, z))
    print(json.dumps({k: round(v, 4) for k, v in r.items()}), flush=True)
    for P_, K_, Q_, lab in ((25216, 3072, 768, "fc1_dgrad"), (25216, 768, 768, "proj_dgrad"),
                            (25216, 2304, 768, "qkv_dgrad")):
        a = (torch.rand(P_, K_, device="cuda") - 0.5).to(torch.bfloat16)
        b = (torch.rand(K_, Q_, device="cuda") - 0.5).to(torch.bfloat16)
        fl = 2.0 * P_ * K_ * Q_
        o = {"shape": lab}
        for t in (0, 1, 3, 16):
            o[f"t{t}"] = round(fl / timeit(lambda: C.gemm(a, b, True, tile=t)) / 1e9, 1)
        o["blas"] = round(fl / timeit(lambda: a @ b) / 1e9, 1)
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
