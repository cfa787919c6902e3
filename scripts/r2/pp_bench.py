"""Ping-pong GEMM tiles (gemm_pp.hip) vs the gemm.hip tiles and torch (hipBLASLt):
correctness (rel err vs fp32) and time per shape / orientation."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from torchbooster_amd.ops._ext import native

SHAPES = [(4096, 4096, 4096, "sq4k"), (8192, 8192, 8192, "sq8k"),
          (25216, 2304, 768, "vit_qkv"), (25216, 768, 768, "vit_proj"), (25216, 3072, 768, "vit_fc1"),
          (25216, 768, 3072, "vit_fc2"), (50176, 1024, 256, "r50_l3_expand"), (50176, 256, 1024, "r50_l3_reduce"),
          (12544, 2048, 512, "r50_l4_expand"), (12544, 512, 2048, "r50_l4_reduce"), (200704, 512, 128, "r50_l2_expand")]
TILES = [0, 1, 2, 3, 13] + list(range(16, 16 + 5))


def timeit(fn, reps=10):
    for _ in range(2):
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
    assert C.gemm_num_tiles() == 21, C.gemm_num_tiles()
    for P, Q, K, lab in SHAPES:
        x = torch.randn(P, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Q, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        wt = w.t().contiguous()
        fl = 2.0 * P * Q * K
        ref = (x[:512].float() @ w.float().t())
        for tw, wa in ((False, w), (True, wt)):
            t_torch = timeit(lambda: x @ (wt if tw else w.t()))
            res = {}
            for tile in TILES:
                y = C.gemm(x, wa, tw, tile=tile)[0]
                err = ((y[:512].float() - ref).norm() / ref.norm()).item()
                ms = timeit(lambda: C.gemm(x, wa, tw, tile=tile))
                res[tile] = (round(ms, 4), round(fl / ms / 1e9, 1), round(err, 5))
            best = min(res, key=lambda t: res[t][0])
            print(json.dumps({"shape": lab, "tw": tw, "torch_ms": round(t_torch, 4),
                              "torch_tf": round(fl / t_torch / 1e9, 1), "best": best, "res": res}), flush=True)
            bad = [t for t, r in res.items() if r[2] > 1e-2]
            assert not bad, (lab, tw, bad, res)


if __name__ == "__main__":
    main()
