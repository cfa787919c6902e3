"""Parallelism: native bucketed data parallel over RCCL / xGMI (the only strategy the reference has)."""
from torchbooster_amd.parallel.ddp import DistributedDataParallel, live_wrappers, no_sync_all, zero_grad_params

DDP = DistributedDataParallel
