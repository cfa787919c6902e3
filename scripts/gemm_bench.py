"""Time the native GEMM engine against torch (hipBLASLt) on the framework's shapes.
Prints one JSON line per (shape, orientation): best native tile, ms, TF/s, torch ms."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from torchbooster_amd.ops._ext import native

SHAPES = [  # (P, Q, K, label)
    (4096, 4096, 4096, "square4k"),
    (25216, 2304, 768, "vit_qkv"), (25216, 768, 768, "vit_proj"), (25216, 3072, 768, "vit_fc1"),
    (25216, 768, 3072, "vit_fc2"),
    (802816, 256, 64, "r50_l1_expand"), (802816, 64, 256, "r50_l1_reduce"), (200704, 512, 128, "r50_l2_expand"),
    (200704, 128, 512, "r50_l2_reduce"), (50176, 1024, 256, "r50_l3_expand"), (50176, 256, 1024, "r50_l3_reduce"),
    (12544, 2048, 512, "r50_l4_expand"), (12544, 512, 2048, "r50_l4_reduce"),
    (256, 512, 768, "mlp_784"), (256, 1000, 2048, "fc_head"),
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
    for P, Q, K, lab in SHAPES:
        x = torch.randn(P, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(Q, K, device="cuda").to(torch.bfloat16)
        wt = w.t().contiguous()
        fl = 2.0 * P * Q * K
        t_torch = timeit(lambda: x @ w.t())
        t_torch_nn = timeit(lambda: x @ wt)
        # weight gradient dW = dyᵀ x (reduction over the P rows), split-K
        dy = torch.randn(P, Q, device="cuda").to(torch.bfloat16)
        t_tw = timeit(lambda: dy.t() @ x)
        resw = {}
        for tile in range(C.gemm_num_tiles()):
            try:
                resw[tile] = timeit(lambda: C.gemm(dy, x, True, tx=True, tile=tile, splits=0))
            except Exception:  # noqa: BLE001
                resw[tile] = float("inf")
        bw = min(resw, key=resw.get)
        print(json.dumps({"shape": lab, "P": P, "Q": Q, "K": K, "wgrad": True, "best_tile": bw,
                          "ms": round(resw[bw], 4), "tflops": round(fl / resw[bw] / 1e9, 1),
                          "torch_ms": round(t_tw, 4), "torch_tflops": round(fl / t_tw / 1e9, 1),
                          "all_ms": {k: round(v, 4) for k, v in resw.items()}}), flush=True)
        for tw, wa in ((False, w), (True, wt)):
            res = {}
            for tile in range(C.gemm_num_tiles()):
                try:
                    res[tile] = timeit(lambda: C.gemm(x, wa, tw, tile=tile))
                except Exception as e:  # noqa: BLE001
                    res[tile] = float("inf")
            best = min(res, key=res.get)
            heur = C.gemm_pick_tile(P, Q, K)
            print(json.dumps({"shape": lab, "P": P, "Q": Q, "K": K, "tw": tw, "best_tile": best,
                              "ms": round(res[best], 4), "tflops": round(fl / res[best] / 1e9, 1),
                              "heur_tile": heur, "heur_ms": round(res[heur], 4),
                              "torch_ms": round(t_torch_nn if tw else t_torch, 4),
                              "torch_tflops": round(fl / (t_torch_nn if tw else t_torch) / 1e9, 1),
                              "all_ms": {k: round(v, 4) for k, v in res.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
