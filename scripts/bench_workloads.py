"""Secondary BASELINE.json workloads, native vs the stock PyTorch-ROCm stack (1 GPU).

  python scripts/bench_workloads.py --workload dcgan   # DCGAN-128 G/D step (two optimizers), bf16
  python scripts/bench_workloads.py --workload nst     # VGG-19 offline style transfer @512, pixels optimised
  python scripts/bench_workloads.py --workload vit     # ViT-B/16 224 px (delegates to bench.py --model vit_b_16)

``--mode native`` runs this framework (bf16 NHWC, native conv/BN/attention/
optimizer kernels); ``--mode stock`` runs the same model definitions on stock
ATen/MIOpen under autocast (``TBAMD_FORCE_REFERENCE=1``), ``torch.optim.AdamW``.
``--mode stock32`` (nst only) is the reference's own precision (fp32, no autocast,
examples/img_stt/offline/offline.yml).  Synthetic data, random-init weights.
One JSON line per run.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _timeit(step, warmup, steps):
    import torch

    for i in range(warmup):
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        print(f"[bench] warmup {i + 1}/{warmup} {time.perf_counter() - t:.2f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, out


def dcgan(a):
    import torch
    import torch.nn.functional as F

    from torchbooster_amd import utils
    from torchbooster_amd.models import DCGANDiscriminator, DCGANGenerator

    dev = torch.device("cuda")
    torch.manual_seed(0)
    G = DCGANGenerator(128, 64).to(dev).to(memory_format=torch.channels_last)
    D = DCGANDiscriminator(64).to(dev).to(memory_format=torch.channels_last)
    B = a.batch
    X = (torch.rand(B, 3, 128, 128, device=dev) * 2 - 1).contiguous(memory_format=torch.channels_last)
    if a.mode == "native":
        from torchbooster_amd.ops.optim import FusedAdamW

        G, D, X = G.to(torch.bfloat16), D.to(torch.bfloat16), X.to(torch.bfloat16)
        go, do = FusedAdamW(G.parameters(), lr=2e-4, betas=(0.5, 0.999)), FusedAdamW(D.parameters(), lr=2e-4,
                                                                                       betas=(0.5, 0.999))
        ctx = torch.autocast("cuda", enabled=False)
    else:
        go = torch.optim.AdamW(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
        do = torch.optim.AdamW(D.parameters(), lr=2e-4, betas=(0.5, 0.999))
        ctx = torch.autocast("cuda", dtype=torch.bfloat16)

    def step():
        with ctx:
            z = torch.randn(B, 128, device=dev, dtype=X.dtype)
            fake = G(z)
            d_loss = F.softplus(-D(X)).float().mean() + F.softplus(D(fake.detach())).float().mean()
        utils.step(d_loss, do)
        # native: the G step runs under utils.frozen(D) as examples/img_gen/dcgan does -- D's weight
        # gradients of the G loss are discarded by the next D step's zero_grad in the reference
        # loop (gan.py:102-113) anyway, so skipping them changes no update
        with ctx, (utils.frozen(D) if a.mode == "native" else contextlib.nullcontext()):
            g_loss = F.softplus(-D(fake)).float().mean()
            utils.step(g_loss, go)
        return g_loss.detach()

    if a.graph and a.mode == "native":  # both optimizer steps in one replayed graph
        step = utils.GraphedStep(step, [do, go], [], warmup=3)
    dt, loss = _timeit(step, a.warmup, a.steps)
    return {"metric": "DCGAN-128 G+D training steps/s (1 GPU)", "value": round(1 / dt, 3), "unit": "steps/s",
            "images_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 3), "batch": B,
            "final_g_loss": float(loss)}


def nst(a):
    import torch

    from torchbooster_amd import utils
    from torchbooster_amd.models.style import gram_matrix_flat, total_variation
    from torchbooster_amd.models.vgg import vgg19

    dev = torch.device("cuda")
    torch.manual_seed(0)
    dtype = torch.bfloat16 if a.mode in ("native", "stock") else torch.float32
    vgg = vgg19().features.to(dev).to(memory_format=torch.channels_last).eval()
    if a.mode == "native":
        vgg = vgg.to(torch.bfloat16)
    native = a.mode in ("native", "native32")
    utils.freeze(vgg)
    S = a.size
    style_layers, content_layers = [0, 5, 10, 19, 28], [29]
    sw = [1.0, 0.8, 0.5, 0.3, 0.1]
    feats = {}

    def hook(i):
        def f(m, inp, out):
            feats[i] = out
        return f

    for l in set(style_layers + content_layers):
        vgg[l].register_forward_hook(hook(l))
    ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=(a.mode == "stock"))
    g = torch.Generator(device=dev).manual_seed(1)
    style = torch.rand(1, 3, S, S, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    content = torch.rand(1, 3, S, S, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    in_dt = torch.bfloat16 if a.mode == "native" else torch.float32
    with torch.no_grad(), ac:
        vgg(style.to(in_dt))
        s_grams = [gram_matrix_flat(feats[l]).float() for l in style_layers]
        vgg(content.to(in_dt))
        c_feats = [feats[l].float() for l in content_layers]
    mixture = content.clone().requires_grad_(True)
    if native:
        from torchbooster_amd.ops.optim import FusedAdamW

        opt = FusedAdamW([mixture], lr=0.1, weight_decay=1e-6)
    else:
        opt = torch.optim.AdamW([mixture], lr=0.1, weight_decay=1e-6)

    def step():
        with ac:
            vgg(mixture.to(in_dt))
            s_loss = sum(w * (gram_matrix_flat(feats[l]).float() - gg).pow(2).mean()
                         for w, l, gg in zip(sw, style_layers, s_grams))
            c_loss = sum((feats[l].float() - c).pow(2).mean() for l, c in zip(content_layers, c_feats))
            loss = 1e6 * s_loss + c_loss + 1e-6 * total_variation(mixture)
        utils.step(loss, opt)
        return loss.detach()

    if a.graph and native:
        step = utils.GraphedStep(step, [opt], [], warmup=2)
    dt, loss = _timeit(step, a.warmup, a.steps)
    return {"metric": f"VGG-19 offline style transfer @{S} iterations/s (1 GPU)", "value": round(1 / dt, 3),
            "unit": "iter/s", "ms_per_step": round(dt * 1e3, 3), "compute_dtype": str(dtype).replace("torch.", ""),
            "final_loss": float(loss)}


def online(a):
    """E6 (examples/img_stt/online/online.py:128-158, online.yml): StyleNet training step
    against a frozen VGG-16 loss network, b8 @256 — style Grams precomputed, content
    features, mixture through VGG, Gram + content + TV losses, clip 1, AdamW 1e-5.
    ``--mode native32`` / ``stock32`` run the reference's fp32; ``native`` / ``stock``
    bf16 (stock: autocast)."""
    import torch
    import torch.nn.functional as F

    from torchbooster_amd import utils
    from torchbooster_amd.models.style import StyleNet, gram_matrix, total_variation
    from torchbooster_amd.models.vgg import vgg16

    dev = torch.device("cuda")
    torch.manual_seed(0)
    native = a.mode in ("native", "native32")
    dt = torch.bfloat16 if a.mode == "native" else torch.float32
    vgg = utils.freeze(vgg16().features.to(dev).to(memory_format=torch.channels_last).eval().to(dt))
    net = StyleNet().to(dev).to(memory_format=torch.channels_last).to(dt)
    layers, cl = [3, 8, 15, 22], 15
    feats = {}
    for l in set(layers + [cl]):
        vgg[l].register_forward_hook(lambda m, i, o, l=l: feats.__setitem__(l, o))
    ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=(a.mode == "stock"))
    S, B = a.size, a.batch
    g = torch.Generator(device=dev).manual_seed(1)
    style = torch.rand(1, 3, S, S, device=dev, generator=g).contiguous(memory_format=torch.channels_last).to(dt)
    content = torch.rand(B, 3, S, S, device=dev, generator=g).contiguous(memory_format=torch.channels_last).to(dt)
    with torch.no_grad(), ac:
        vgg(style)
        s_grams = [gram_matrix(feats[l]).float() for l in layers]
    if native:
        from torchbooster_amd.ops.optim import FusedAdamW

        opt = FusedAdamW(net.parameters(), lr=1e-5, weight_decay=1e-2)
    else:
        opt = torch.optim.AdamW(net.parameters(), lr=1e-5, weight_decay=1e-2)

    def step():
        with ac:
            with torch.no_grad():
                vgg(content)
                c_feat = feats[cl].float()
            mixture = net(content)
            vgg(mixture)
            m_grams = [gram_matrix(feats[l]).float() for l in layers]
            s_loss = sum(F.mse_loss(m, s.expand_as(m)) for m, s in zip(m_grams, s_grams))
            c_loss = F.mse_loss(feats[cl].float(), c_feat)
            loss = 1e5 * s_loss + c_loss + 1e-6 * total_variation(mixture).float()
        utils.step(loss, opt, clip=1.0)
        return loss.detach()

    sec, loss = _timeit(step, a.warmup, a.steps)
    return {"metric": f"online style transfer (StyleNet + VGG-16 loss) b{B} @{S} iterations/s (1 GPU)",
            "value": round(1 / sec, 3), "unit": "iter/s", "ms_per_step": round(sec * 1e3, 3),
            "compute_dtype": "bfloat16" if a.mode in ("native", "stock") else "float32", "final_loss": float(loss)}


def adain_wl(a):
    """E7 (examples/img_stt/adain/adain.py:52-80, adain.yml): AdaIN decoder training step at
    b32 @256 — frozen VGG-16 encoder (hooks 3/8/15/22) over style and content, AdaIN at
    relu4_1, decoder, mixture through the encoder, per-layer mean/std style loss (x10) +
    content MSE, clip 1, AdamW 1e-4.  The reference runs it under AMP (``fp16: true``):
    ``native`` = bf16 NHWC on this framework, ``stock`` = the same modules on ATen/MIOpen
    under bf16 autocast; ``native32`` / ``stock32`` = fp32."""
    import torch
    import torch.nn.functional as F

    from torchbooster_amd import utils
    from torchbooster_amd.models.style import AdaINDecoder, adain, mu_std, style_stats_loss
    from torchbooster_amd.models.vgg import vgg16

    dev = torch.device("cuda")
    torch.manual_seed(0)
    native = a.mode in ("native", "native32")
    dt = torch.bfloat16 if a.mode == "native" else torch.float32
    layers = [3, 8, 15, 22]
    enc = utils.freeze(vgg16().features[: max(layers) + 1].to(dev).to(memory_format=torch.channels_last).eval().to(dt))
    dec = AdaINDecoder().to(dev).to(memory_format=torch.channels_last).to(dt)
    feats = {}
    for l in layers:
        enc[l].register_forward_hook(lambda m, i, o, l=l: feats.__setitem__(l, o))
    ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=(a.mode == "stock"))
    S, B = a.size, a.batch
    g = torch.Generator(device=dev).manual_seed(1)
    style = torch.rand(B, 3, S, S, device=dev, generator=g).contiguous(memory_format=torch.channels_last).to(dt)
    content = torch.rand(B, 3, S, S, device=dev, generator=g).contiguous(memory_format=torch.channels_last).to(dt)
    if native:
        from torchbooster_amd.ops.optim import FusedAdamW

        opt = FusedAdamW(dec.parameters(), lr=1e-4, weight_decay=1e-2)
    else:
        opt = torch.optim.AdamW(dec.parameters(), lr=1e-4, weight_decay=1e-2)

    def s_crit(mfs, sfs):
        if native:  # framework loss: same value on [N, C] statistics, no expanded broadcasts
            return style_stats_loss(mfs, sfs)
        return sum(F.mse_loss(xm.float(), sm.float()) + F.mse_loss(xs.float(), ss.float())
                   for (xm, xs), (sm, ss) in zip(map(mu_std, mfs), map(mu_std, sfs)))

    def step():
        with ac:
            with torch.no_grad():
                enc(style)
                s_feats = [feats[l].detach() for l in layers]
                enc(content)
                c_feats = [feats[l].detach() for l in layers]
            mixture = dec(adain(s_feats[-1], c_feats[-1]))
            enc(mixture)
            m_feats = [feats[l] for l in layers]
            loss = 10 * s_crit(m_feats, s_feats) + F.mse_loss(m_feats[-1].float(), c_feats[-1].float())
        utils.step(loss, opt, clip=1.0)
        return loss.detach()

    sec, loss = _timeit(step, a.warmup, a.steps)
    return {"metric": f"AdaIN decoder training (VGG-16 encoder) b{B} @{S} iterations/s (1 GPU)",
            "value": round(1 / sec, 3), "unit": "iter/s", "images_per_s": round(B / sec, 1),
            "ms_per_step": round(sec * 1e3, 3), "compute_dtype": "bfloat16" if a.mode in ("native", "stock") else "float32",
            "final_loss": float(loss)}


def _small_opt(a, params, lr):
    import torch

    if a.mode == "native":
        from torchbooster_amd.ops.optim import FusedAdamW

        return FusedAdamW(params, lr=lr, weight_decay=1e-2)
    return torch.optim.AdamW(params, lr=lr, weight_decay=1e-2)


def _small_step(a, train, opt, sched):
    """Eager step (scheduler stepped after it) or a GraphedStep replay (--graph)."""
    from torchbooster_amd import utils

    if a.graph:
        return utils.GraphedStep(train, [opt], [sched], warmup=2)

    def step(*inputs):
        out = train(*inputs)
        sched.step()
        return out

    return step


def lenet(a):
    """E1 (examples/img_cls/lenet/lenet.py:51-75): MNIST-shape LeNet step, b256."""
    import torch

    from torchbooster_amd import models, utils
    from torchbooster_amd.ops.loss import cross_entropy_accuracy
    from torchbooster_amd.scheduler import CycleScheduler

    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = a.batch
    model = models.lenet(10).to(dev).to(memory_format=torch.channels_last)
    X = torch.randn(B, 1, 28, 28, device=dev).contiguous(memory_format=torch.channels_last)
    Y = torch.randint(0, 10, (B,), device=dev)
    dt = torch.bfloat16 if a.mode == "native" else torch.float32
    model, X = model.to(dt), X.to(dt)
    opt = _small_opt(a, model.parameters(), 3e-4)
    sched = CycleScheduler(opt, 3e-4, a.warmup + a.steps + 10, warmup=2)
    ctx = torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.mode != "native")

    def train(x, y):
        with ctx:
            loss, acc = cross_entropy_accuracy(model(x), y)
        utils.step(loss, opt)
        return loss.detach()

    step = _small_step(a, train, opt, sched)
    dt_, loss = _timeit(lambda: step(X, Y), a.warmup, a.steps)
    return {"metric": "LeNet MNIST training steps/s (1 GPU)", "value": round(1 / dt_, 2), "unit": "steps/s",
            "images_per_s": round(B / dt_, 1), "ms_per_step": round(dt_ * 1e3, 4), "batch": B,
            "final_loss": float(loss)}


def vae(a):
    """E4 (examples/img_gen/vae/vae.py:100-120): MLP VAE step, b256, KL weight 2.5e-4, clip 1."""
    import torch
    import torch.nn.functional as F

    from torchbooster_amd import models, utils
    from torchbooster_amd.ops.losses import bce_with_logits, gaussian_kld
    from torchbooster_amd.scheduler import CycleScheduler

    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = a.batch
    model = models.VAE(128).to(dev)
    X = torch.rand(B, 1, 28, 28, device=dev)
    dt = torch.bfloat16 if a.mode == "native" else torch.float32
    model, X = model.to(dt), X.to(dt)
    opt = _small_opt(a, model.parameters(), 1e-3)
    sched = CycleScheduler(opt, 1e-3, a.warmup + a.steps + 10, warmup=2)
    ctx = torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.mode != "native")

    def train(x):
        with ctx:
            rec, mu, log_var = model(x)
            bce = bce_with_logits(rec, x)
            kld = gaussian_kld(mu, log_var)
            loss = bce + 2.5e-4 * kld
        utils.step(loss, opt, clip=1.0)
        return loss.detach()

    step = _small_step(a, train, opt, sched)
    dt_, loss = _timeit(lambda: step(X), a.warmup, a.steps)
    return {"metric": "VAE MNIST training steps/s (1 GPU)", "value": round(1 / dt_, 2), "unit": "steps/s",
            "images_per_s": round(B / dt_, 1), "ms_per_step": round(dt_ * 1e3, 4), "batch": B,
            "final_loss": float(loss)}


def cifar(a):
    """E2 (examples/img_cls/resnet/resnet.py:44-68 + resnet.yml): ResNet-18 on CIFAR-10
    shapes at b2048 — AdamW 1e-3, clip 1.0, label smoothing 0.1, CycleScheduler.
    ``--loader device``: every step draws its batch from the HBM-resident uint8
    dataset (50k synthetic images) through the full reference transform on the GPU
    (crop pad 4 reflect, flip, rotation 15, RandAugment(2, 9), normalise:
    data.DeviceImageLoader); ``--loader none``: one fixed device batch."""
    import torch
    import torch.nn.functional as F

    from torchbooster_amd import models, utils
    from torchbooster_amd.scheduler import CycleScheduler

    dev = torch.device("cuda", 0)
    B = a.batch
    model = models.resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    loader = None
    if a.mode == "native":
        from torchbooster_amd.ops.loss import cross_entropy_accuracy
        from torchbooster_amd.ops.optim import FusedAdamW

        model = model.to(torch.bfloat16)
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
    sched = CycleScheduler(opt, 1e-3, 10 ** 6, warmup=240, decay=("lin", "cos"))
    x0 = torch.randn(B, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    y0 = torch.randint(0, 10, (B,), device=dev)
    if a.mode == "native":
        x0 = x0.to(torch.bfloat16)
    if a.loader == "device":
        from torchbooster_amd.config import LoaderConfig
        from torchbooster_amd.data import DeviceAugment, SyntheticImageDataset

        ds = SyntheticImageDataset(50000, (3, 32, 32), 10, transform=DeviceAugment(
            size=32, padding=4, hflip=True, rotate=15, randaugment=True, mean=(0.4914, 0.4822, 0.4465),
            std=(0.2023, 0.1994, 0.2010), dtype=torch.bfloat16 if a.mode == "native" else torch.float32))
        loader = LoaderConfig(batch_size=B, drop_last=True).make(ds, shuffle=True)
        it = [iter(loader)]

    def batch():
        if loader is None:
            return x0, y0
        try:
            return next(it[0])
        except StopIteration:
            it[0] = iter(loader)
            return next(it[0])

    def step():
        x, y = batch()
        if a.mode == "native":
            loss, _ = cross_entropy_accuracy(model(x), y, 0.1)
            utils.step(loss, opt, sched, clip=1.0)
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(model(x), y, label_smoothing=0.1)
            utils.step(loss, opt, sched, clip=1.0)
        return loss

    sec, loss = _timeit(step, a.warmup, a.steps)
    res = {"model": "resnet18-cifar10", "batch": B, "loader": a.loader, "ms_per_step": round(sec * 1e3, 3),
           "img_s": round(B / sec, 1), "final_loss": float(loss)}
    if loader is not None:  # the input pipeline alone
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for x, y in loader:
            n += x.shape[0]
            if n >= 20 * B:
                break
        torch.cuda.synchronize()
        res["loader_only_img_s"] = round(n / (time.perf_counter() - t0), 1)
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["dcgan", "nst", "vit", "lenet", "vae", "cifar", "online", "adain"], required=True)
    ap.add_argument("--loader", choices=["none", "device"], default="none", help="cifar: input pipeline")
    ap.add_argument("--graph", action="store_true", help="replay the whole step as one hipGraph (native mode)")
    ap.add_argument("--mode", choices=["native", "native32", "stock", "stock32"], default="native")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--save-routes", default="", help="write the conv autotune table here afterwards")
    a = ap.parse_args()
    if a.workload == "vit":
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", "vit_b_16", "--batch", str(a.batch),
               "--steps", str(a.steps), "--warmup", str(a.warmup), "--mode",
               "stock" if a.mode != "native" else "native"]
        return subprocess.call(cmd)
    if a.mode not in ("native", "native32"):
        os.environ["TBAMD_FORCE_REFERENCE"] = "1"
    import torch

    from torchbooster_amd import utils

    utils.boost(True)
    res = {"dcgan": dcgan, "nst": nst, "lenet": lenet, "vae": vae, "cifar": cifar, "online": online,
           "adain": adain_wl}[a.workload](a)
    res.update({"workload": a.workload, "mode": a.mode, "graph": a.graph, "steps": a.steps, "warmup": a.warmup, "n_gpus": 1,
                "data": "synthetic, random-init weights", "device": torch.cuda.get_device_name()})
    print(json.dumps(res), flush=True)
    if a.save_routes:
        from torchbooster_amd.ops.conv import save_routes

        save_routes(a.save_routes)
    return 0


if __name__ == "__main__":
    sys.exit(main())
