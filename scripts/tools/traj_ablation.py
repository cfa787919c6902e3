"""ResNet-18 (torchvision layout) CIFAR b256, 20 steps from one init over the same batches
(tests/test_gpu_trajectory.py): which stage makes the native path's loss curve drift from fp32
further than stock bf16?  Prints one JSON line per variant: mean |loss - fp32 loss| over the steps.

  fp32            stock ATen fp32 + torch AdamW (the truth)
  autocast[i]     stock autocast bf16 over fp32 params + torch AdamW (3 reruns)
  pure            stock model in bf16 + torch AdamW on the bf16 params
  pure_fused      stock model in bf16 (ATen kernels) + FusedAdamW (fp32 master weights)
  native          nativize(bf16) + FusedAdamW                      (the tested path)
  native_rerun    the same again (run-to-run spread of the native path)
  native_torchopt nativize(bf16) fwd/bwd + torch AdamW on fp32 master copies
  native_nofuse   nativize(bf16, fuse=False): native leaf kernels, no cross-layer links
  native_f32res   native, but every BasicBlock's residual add + ReLU in fp32 (ATen) after the BN
"""
import copy
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.nativize import nativize  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

STEPS = int(os.environ.get("STEPS", "20"))
bf = torch.bfloat16


def batches(n, B, img, classes, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [(torch.randn(B, 3, img, img, device="cuda", generator=g),
             torch.randint(0, classes, (B,), device="cuda", generator=g)) for _ in range(n)]


def train(model, data, step_fn, dtype=None, autocast=False):
    losses = []
    for i in range(STEPS):
        x, y = data[i % len(data)]
        x = x.contiguous(memory_format=torch.channels_last)
        if dtype is not None:
            x = x.to(dtype)
        with torch.autocast("cuda", dtype=bf, enabled=autocast):
            out = model(x)
        loss = F.cross_entropy(out.float(), y)
        step_fn(loss)
        losses.append(loss.item())
    return torch.tensor(losses)


def opt_step(opt):
    def f(loss):
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    return f


def master_step(model):
    ps = list(model.parameters())
    ms = [p.detach().float().clone().requires_grad_() for p in ps]
    opt = torch.optim.AdamW(ms, lr=1e-3)

    def f(loss):
        for p in ps:
            p.grad = None
        loss.backward()
        for p, m in zip(ps, ms):
            m.grad = p.grad.float()
        opt.step()
        with torch.no_grad():
            for p, m in zip(ps, ms):
                p.copy_(m)
    return f


def f32_residual(model):
    """Every BasicBlock: conv/BN native, the residual add + ReLU in fp32."""
    def fwd(blk, x):
        from torchbooster_amd.models.resnet import conv_bn_act
        h = conv_bn_act(blk.conv1, blk.bn1, x, "relu")
        z = conv_bn_act(blk.conv2, blk.bn2, h, "none")
        idt = x if blk.downsample is None else conv_bn_act(blk.downsample[0], blk.downsample[1], x, "none")
        return (z.float() + idt.float()).relu().to(x.dtype)
    import types
    for m in model.modules():
        if type(m).__name__ == "BasicBlock":
            object.__setattr__(m, "forward", types.MethodType(fwd, m))
    # the trunk's fused forward calls blocks through their own forward when they are not linked
    for name in ("_tb_impl",):
        pass
    return model


ONLY = [v for v in os.environ.get("VARIANTS", "").split(",") if v]  # subset (fp32 + autocast always run)


def variants(base, data):
    """(name, loss curve) of every variant on one set of batches."""
    from torchbooster_amd.ops import conv as nconv

    res = {}
    if ONLY:
        return variants_subset(base, data, res)
    m = copy.deepcopy(base)
    res["fp32"] = train(m, data, opt_step(torch.optim.AdamW(m.parameters(), lr=1e-3)))
    for i in range(3):
        m = copy.deepcopy(base)
        res[f"autocast{i}"] = train(m, data, opt_step(torch.optim.AdamW(m.parameters(), lr=1e-3)), autocast=True)
    m = copy.deepcopy(base).to(bf)
    res["pure"] = train(m, data, opt_step(torch.optim.AdamW(m.parameters(), lr=1e-3)), dtype=bf)
    m = copy.deepcopy(base).to(bf)
    res["pure_fused"] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)), dtype=bf)
    m = nativize(copy.deepcopy(base).to(bf))
    res["native"] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)), dtype=bf)
    m = nativize(copy.deepcopy(base).to(bf))
    res["native_torchopt"] = train(m, data, master_step(m), dtype=bf)
    m = nativize(copy.deepcopy(base).to(bf), fuse=False)
    res["nofuse"] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)), dtype=bf)
    no_mio = nconv._NO_MIOPEN
    nconv._NO_MIOPEN = False
    for dirs in (("fwd",), ("dgrad",), ("wgrad",), ("fwd", "dgrad", "wgrad")):
        old = dict(nconv._FORCE)
        for d in dirs:
            nconv._FORCE[d] = "miopen"
        m = nativize(copy.deepcopy(base).to(bf), fuse=False)
        res["nofuse_miopen_" + "+".join(dirs)] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)),
                                                       dtype=bf)
        nconv._FORCE.clear()
        nconv._FORCE.update(old)
    nconv._NO_MIOPEN = no_mio
    os.environ["TBAMD_FORCE_REFERENCE"] = "1"
    m = nativize(copy.deepcopy(base).to(bf), fuse=False)
    res["nofuse_all_aten"] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)), dtype=bf)
    del os.environ["TBAMD_FORCE_REFERENCE"]
    return res


def variants_subset(base, data, res):
    m = copy.deepcopy(base)
    res["fp32"] = train(m, data, opt_step(torch.optim.AdamW(m.parameters(), lr=1e-3)))
    for i in range(int(os.environ.get("N_AUTOCAST", "1"))):
        m = copy.deepcopy(base)
        res[f"autocast{i}"] = train(m, data, opt_step(torch.optim.AdamW(m.parameters(), lr=1e-3)), autocast=True)
    if "pure" in ONLY:
        m = copy.deepcopy(base).to(bf)
        res["pure"] = train(m, data, opt_step(torch.optim.AdamW(m.parameters(), lr=1e-3)), dtype=bf)
    if "native" in ONLY:
        m = nativize(copy.deepcopy(base).to(bf))
        res["native"] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)), dtype=bf)
    if "nofuse" in ONLY:
        m = nativize(copy.deepcopy(base).to(bf), fuse=False)
        res["nofuse"] = train(m, data, opt_step(FusedAdamW(m.parameters(), lr=1e-3)), dtype=bf)
    return res


def main():
    torch.manual_seed(0)
    base = models.tv.resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    devs = {}
    seeds = [int(v) for v in os.environ.get("SEEDS", "1,2,3").split(",")]
    for seed in seeds:  # batch sets: the deviation of one trajectory is a chaotic draw
        res = variants(base, batches(4, 256, 32, 10, seed=seed))
        l32 = res["fp32"]
        na = len([k for k in res if k.startswith("autocast")])
        amp = sum((res[f"autocast{i}"] - l32).abs().mean().item() for i in range(na)) / na
        for k, v in res.items():
            d = (v - l32).abs().mean().item()
            devs.setdefault(k, []).append((d, d / amp))
            print(json.dumps({"seed": seed, "variant": k, "dev": round(d, 5), "x_autocast": round(d / amp, 2),
                              "curve": [round(a, 4) for a in v.tolist()]}), flush=True)
    for k, v in devs.items():
        print(json.dumps({"variant": k, "mean_x_autocast": round(sum(r for _, r in v) / len(v), 2),
                          "x_autocast": [round(r, 2) for _, r in v]}), flush=True)


if __name__ == "__main__":
    main()
