"""Probe: can RCCL run a multi-rank group when every rank shares ONE GPU?

The only GPU box available to the builder has one MI355X, so the multi-rank RCCL path of the
native reducer has never run.  This launches WORLD ranks (torch.distributed.run) that all bind
cuda:0 and tries a plain all_reduce, then (if that works) 3 steps of the native DDP reducer on a
small ResNet, checking parameters stay bit-identical across ranks.

Usage (on the GPU box):
    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 scripts/tools/rccl_shared_gpu_probe.py
"""
import os
import sys
import time

import torch
import torch.distributed as tdist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main() -> int:
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from datetime import timedelta

    tdist.init_process_group("nccl", timeout=timedelta(seconds=60), device_id=dev)
    t = torch.full((1 << 20,), float(rank + 1), device=dev)
    tdist.all_reduce(t)
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    ok = bool((t == want).all())
    print(f"[rank {rank}] all_reduce sum over {world} ranks sharing cuda:0: {t[0].item()} (want {want}) ok={ok}",
          flush=True)
    if not ok:
        return 1
    # bandwidth-ish figure for a 97 MiB fp32 buffer (ResNet-50 gradient size); ranks share one
    # device so this is NOT an xGMI number, only proof that the collective runs
    big = torch.ones(25_557_032, device=dev)
    for _ in range(2):
        tdist.all_reduce(big)
    torch.cuda.synchronize()
    tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(5):
        tdist.all_reduce(big)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"[rank {rank}] 97.5 MiB fp32 all_reduce: {dt * 1e3:.2f} ms (shared device)", flush=True)

    from torchbooster_amd import models, utils
    from torchbooster_amd.ops.loss import cross_entropy_accuracy
    from torchbooster_amd.ops.optim import FusedAdamW
    from torchbooster_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    model = models.resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    ddp = DistributedDataParallel(model, bucket_cap_mb=4.0)
    opt = FusedAdamW(ddp.parameters(), lr=1e-3, weight_decay=1e-2)
    g = torch.Generator(device="cpu").manual_seed(100 + rank)  # different data per rank
    for _ in range(3):
        x = torch.randn(8, 3, 64, 64, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), generator=g).to(dev)
        loss, _ = cross_entropy_accuracy(ddp(x), y, 0.1)
        utils.step(loss, opt, clip=1.0)
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().float().flatten() for p in model.parameters()])
    ref = flat.clone()
    tdist.broadcast(ref, 0)
    same = bool(torch.equal(flat, ref))
    print(f"[rank {rank}] native DDP reducer over RCCL, 3 AdamW steps, params identical to rank 0: {same} "
          f"loss={loss.item():.4f}", flush=True)
    tdist.destroy_process_group()
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
