"""Headline benchmark: ResNet-50 224px bf16 data-parallel training, images/s (whole job).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1
it is launched by ``torch.distributed.run`` with one rank per GPU (RCCL).  W
untimed warmup steps, then exactly K timed steps bracketed by barrier +
device synchronize; the slowest rank's time is reported.  Rank 0 prints one
JSON line.

A timed step is the reference's full training step (utils.step,
/root/reference/torchbooster/utils.py:204-252, as driven by
/root/reference/examples/img_cls/resnet/resnet.py:44-68): forward, label-
smoothed cross-entropy, backward with the bucketed gradient all-reduce, global
grad-norm clip (1.0), AdamW (lr 1e-3, wd 1e-2) and the CycleScheduler step.
Data: synthetic images/labels of the ImageNet shape resident on the device;
weights: random init (no network in this environment).

``--mode native`` (default) runs this framework's MI355X path.  ``--mode
stock`` runs the reference stack on the same model and data (ATen/MIOpen
BatchNorm+ReLU+add, autocast bf16 over f32 params, torch.optim.AdamW,
torch DDP over RCCL) — the comparator recorded in BASELINE.md.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

# measured comparator (stock PyTorch-ROCm stack, this script --mode stock, 1x MI355X,
# b256/GPU); see BASELINE.md.  Used for vs_baseline (x N for N GPUs: linear weak-
# scaling of the measured 1-GPU number, i.e. a conservative ratio).
STOCK_1GPU_IMG_S = None
_LABEL = {"resnet50": "ResNet-50", "stock_resnet50": "ResNet-50 (stock nn + nativize)", "resnet18": "ResNet-18", "vit_b_16": "ViT-B/16", "vit_s_16": "ViT-S/16"}


def _load_stock_baseline():
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "stock_baseline.json")
    try:
        with open(p) as f:
            return float(json.load(f)["img_s_1gpu"])
    except Exception:
        return STOCK_1GPU_IMG_S


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU).  Without torchrun's WORLD_SIZE, N > 1 spawns the N ranks itself "
                         "through torchbooster_amd.distributed.launch")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--mode", choices=["native", "stock"], default="native")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--ddp", action="store_true",
                    help="wrap in the native DDP reducer even at N=1 (a 1-rank RCCL group, every bucket "
                         "all-reduced): measures the wrapper's overhead on hardware")
    ap.add_argument("--reduce-dtype", choices=["grad", "fp32"], default="grad",
                    help="all-reduce dtype: the grad dtype (bf16) or f32 accumulation")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="off",
                    help="replay the whole native step (fwd, bwd, all-reduce, clip, AdamW) as one hipGraph "
                         "(utils.GraphedStep; auto = on for a single rank).  Off by default: the eager ResNet-50 "
                         "step is GPU-bound (22.5 ms eager vs 22.9 ms replayed, profiles/r02_lmdb)")
    return ap


def main() -> int:
    a = _parser().parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world}; refusing to report a number for the "
              "wrong world size", file=sys.stderr)
        return 2
    if env_world is None and a.gpus > 1:
        # no torchrun: spawn one rank per GPU ourselves (the framework launcher,
        # reference distributed.py:130-153).  Nothing in this parent touches the GPU.
        import torchbooster_amd.distributed as dist

        backend = os.environ.get("TBAMD_BENCH_BACKEND", "nccl")
        dist.launch(_rank_main, a.gpus, args=(vars(a),), backend=backend)
        return 0
    return _rank_main(vars(a))


def _rank_main(opts: dict) -> int:
    a = argparse.Namespace(**opts)
    # native libraries write to fd 1 (RCCL prints its version banner when a communicator comes up):
    # the run's stdout goes to stderr, and the one JSON line goes to the real stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if a.mode == "stock":
        os.environ["TBAMD_FORCE_REFERENCE"] = "1"
        os.environ.setdefault("TBAMD_GEMM_TABLE", "none")  # the reference stack: heuristic GEMM picks
    os.environ.setdefault("TBAMD_TUNE_LOG", "1")
    import torch
    import torch.distributed as tdist
    import torch.nn.functional as F

    import torchbooster_amd.distributed as dist
    from torchbooster_amd import models, utils
    from torchbooster_amd.ops.loss import cross_entropy_accuracy
    from torchbooster_amd.scheduler import CycleScheduler

    # a rank spawned by dist.launch arrives with its process group initialised;
    # a torchrun rank has RANK / WORLD_SIZE in the environment
    world = tdist.get_world_size() if tdist.is_initialized() else int(os.environ.get("WORLD_SIZE", "1"))
    # TBAMD_BENCH_BACKEND=gloo: multi-rank rehearsal of the DDP path on a box with fewer
    # GPUs than ranks (ranks share devices round-robin); the driver's runs use RCCL
    backend = os.environ.get("TBAMD_BENCH_BACKEND", "nccl")
    if world == 1 and a.ddp:  # 1-rank process group so the reducer's collective path runs
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(dist.find_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("LOCAL_RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if (world > 1 or a.ddp) and not tdist.is_initialized():
        dist.init_from_env(backend)
    local = dist.get_local_rank() if tdist.is_initialized() else int(os.environ.get("LOCAL_RANK", "0"))
    if "LOCAL_RANK" in os.environ:
        local = int(os.environ["LOCAL_RANK"])
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rank = dist.get_rank()
    utils.boost(True)
    torch.manual_seed(1234 + rank)

    stock_model = a.model.startswith("stock_")
    if stock_model:
        # a stock-nn torchvision-layout model (what the reference hands to conf.env.make,
        # resnet.py:111-112 -> config.py:174-178); the native mode puts it on the native
        # kernels through nativize(), exactly as EnvironementConfig.make does
        model = getattr(models.tv, a.model[len("stock_"):])(num_classes=1000)
    else:
        model = getattr(models, a.model)(num_classes=1000)
    model = model.to(dev).to(memory_format=torch.channels_last)
    B, S = a.batch, a.image
    x = torch.randn(B, 3, S, S, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)
    n_iter = a.warmup + a.steps + 10

    if a.mode == "native":
        from torchbooster_amd.ops.optim import FusedAdamW
        from torchbooster_amd.parallel import DistributedDataParallel

        model = model.to(torch.bfloat16)
        x = x.to(torch.bfloat16)
        if stock_model:
            from torchbooster_amd.nativize import nativize

            model = nativize(model)
        ddp = None
        if world > 1 or a.ddp:
            ddp = model = DistributedDataParallel(
                model, bucket_cap_mb=a.bucket_mb, force_reduce=a.ddp,
                reduce_dtype=torch.float32 if a.reduce_dtype == "fp32" else None)
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
        sched = CycleScheduler(opt, 1e-3, n_iter, warmup=max(1, n_iter // 10), decay=("lin", "cos"))

        use_graph = a.graph == "on" or (a.graph == "auto" and world == 1 and not a.ddp)

        def train():
            logits = model(x)
            loss, acc = cross_entropy_accuracy(logits, y, 0.1)
            utils.step(loss, opt, None, clip=1.0)
            return loss

        if use_graph:
            # every kernel of the step replayed from one graph: no per-kernel launch gaps
            graphed = utils.GraphedStep(train, [opt], [sched], warmup=3)

            def step():
                return graphed()
        else:
            def step():
                loss = train()
                sched.step()
                return loss
    else:
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
        sched = CycleScheduler(opt, 1e-3, n_iter, warmup=max(1, n_iter // 10), decay=("lin", "cos"))

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = model(x)
                loss = F.cross_entropy(logits, y, label_smoothing=0.1)
            utils.step(loss, opt, sched, clip=1.0)
            return loss

    if a.mode != "native":
        ddp = None
    model.train()
    # (the caller's stream is the compute stream; the native backward puts its weight gradients on
    # a LOW-priority side stream, ops/streams.py side_stream.  TBAMD_BENCH_HIPRI=1: the whole loop
    # inside streams.step_priority instead -- the round-4 arrangement, kept for A/B runs)
    if a.mode == "native" and os.environ.get("TBAMD_BENCH_HIPRI", "0") == "1":
        from torchbooster_amd.ops import streams as _streams

        run_ctx = _streams.step_priority()
    else:
        run_ctx = contextlib.nullcontext()
    run_ctx.__enter__()
    for i in range(a.warmup):
        tw = time.perf_counter()
        step()
        torch.cuda.synchronize()
        if rank == 0:  # progress (first steps autotune conv routing)
            print(f"[bench] warmup {i + 1}/{a.warmup} {time.perf_counter() - tw:.2f}s", file=sys.stderr, flush=True)
    dist.synchronize()
    # TBAMD_BENCH_STEPTIMES=1 (diagnostic): an event after every timed step, per-step spread on stderr
    # (uniform 18.9-19.3 ms on the headline config, gc.freeze() changes nothing: profiles/r06_host/)
    step_ev = [] if os.environ.get("TBAMD_BENCH_STEPTIMES", "0") == "1" else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if step_ev is not None:
        step_ev.append(torch.cuda.Event(enable_timing=True))
        step_ev[-1].record()
    for _ in range(a.steps):
        loss = step()
        if step_ev is not None:
            step_ev.append(torch.cuda.Event(enable_timing=True))
            step_ev[-1].record()
    t_host = time.perf_counter() - t0  # host submission time: ~elapsed when the step is host-bound
    torch.cuda.synchronize()
    if step_ev is not None and rank == 0:
        seq = [step_ev[i].elapsed_time(step_ev[i + 1]) for i in range(len(step_ev) - 1)]
        dts = sorted(seq)
        print(f"[bench] per-step ms: min {dts[0]:.3f} median {dts[len(dts) // 2]:.3f} max {dts[-1]:.3f} "
              f"in order {' '.join(f'{d:.2f}' for d in seq)}; device memory allocated "
              f"{torch.cuda.memory_allocated(dev) / 2**30:.2f} GiB, peak {torch.cuda.max_memory_allocated(dev) / 2**30:.2f} GiB",
              file=sys.stderr, flush=True)
    dist.synchronize()
    elapsed = time.perf_counter() - t0
    run_ctx.__exit__(None, None, None)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    lv = float(loss.item())
    ms = elapsed / a.steps * 1e3
    img_s = B * world * a.steps / elapsed
    base = _load_stock_baseline()
    vs = None
    if base and a.mode == "native" and a.model == "resnet50" and S == 224 and B == 256:
        vs = img_s / (base * world)
    out = {
        "metric": f"images/sec (whole node) {_LABEL.get(a.model, a.model)} {S}px bf16 DDP",
        "value": round(img_s, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if vs is None else round(vs, 4),
        "dtype": "bf16",
        "data": "synthetic (device-resident random images/labels, random-init weights)",
        "config": {
            "model": a.model,
            "image": S,
            "per_gpu_batch": B,
            "global_batch": B * world,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "ddp_wrapper": ("native" if a.mode == "native" else "torch") if (world > 1 or a.ddp) else None,
            "hip_graph": bool(a.mode == "native" and (a.graph == "on" or (a.graph == "auto" and world == 1
                                                                          and not a.ddp))),
            "reduce_dtype": a.reduce_dtype if a.mode == "native" and (world > 1 or a.ddp) else None,
            "mode": a.mode,
            # what the process group actually is (not what was asked for)
            "backend": tdist.get_backend() if tdist.is_available() and tdist.is_initialized() else None,
            "pg_world_size": tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1,
            "optimizer": "AdamW lr1e-3 wd1e-2 + clip 1.0 + CycleScheduler",
            "loss": "cross_entropy label_smoothing=0.1",
        },
        "baseline_note": "vs_baseline = value / (n_gpus x measured 1-GPU stock PyTorch-ROCm img/s, "
                         "profiles/stock_baseline.json)",
        "final_loss": lv,
    }
    if ddp is not None and getattr(ddp, "precision_probe", False):
        out["ddp_precision"] = ddp.precision_summary()  # low-precision vs f32 bucket reduction
    if rank == 0:
        print(f"[bench] host submit {t_host / a.steps * 1e3:.3f} ms/step vs {ms:.3f} ms/step wall",
              file=sys.stderr, flush=True)
        if a.mode == "native":
            from torchbooster_amd.ops.conv import autotune_table

            tab = autotune_table()
            nat = sum(v == "native" for v in tab.values())
            print(f"[bench] conv routing: {nat}/{len(tab)} (direction, shape) pairs native", file=sys.stderr)
            for k, v in sorted(tab.items(), key=str):
                print(f"[bench]   {v:7s} {k}", file=sys.stderr)
            if a.mode == "native" and ddp is not None:
                print(f"[bench] ddp buckets (MiB): {[round(x, 2) for x in ddp.bucket_sizes_mb()]}", file=sys.stderr)
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if "RANK" in os.environ:  # torchrun / env:// rank: ours to tear down (dist.job tears its own down)
        dist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
