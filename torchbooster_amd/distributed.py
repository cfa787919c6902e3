"""Process-per-GPU runtime over RCCL (reference: /root/reference/torchbooster/distributed.py).

API parity: ``LOCAL_PROCESS_GROUP``, ``get_rank``, ``get_local_rank``,
``get_world_size``, ``is_primary``, ``synchronize``, ``gather``,
``data_sampler``, ``find_free_port``, ``launch``, ``job``.

MI355X design:
* one process per GPU; backend ``"nccl"`` (= RCCL on ROCm, over the xGMI
  mesh) for GPU jobs, ``"gloo"`` for CPU jobs (``n_gpu_per_machine=0`` with
  ``n_proc``, or ``backend="gloo"``) so the whole runtime is testable on CPU;
* the device is bound (``set_device``) BEFORE the first collective (the
  reference's barrier ran before it, putting every rank on GPU 0 — A.2 B9), and
  the NCCL communicator is created eagerly on that device;
* ``torchrun`` / ``env://`` launches are detected and joined in-process;
* ``seed()`` / ``boost()`` state applied in the parent is re-applied inside every
  spawned rank (A.2 B8), with a rank offset available for data RNG;
* ``data_sampler`` honours ``shuffle`` for distributed samplers (A.2 B9) and
  :func:`torchbooster_amd.utils.iter_loader` advances ``set_epoch``.
"""
from __future__ import annotations

import datetime
import logging
import os
import socket
from typing import Any, Callable, List, Optional, Sequence, Tuple

import torch
from torch import distributed as dist
from torch import multiprocessing as mp
from torch.utils.data import Dataset, DistributedSampler, RandomSampler, Sampler, SequentialSampler

__all__ = [
    "LOCAL_PROCESS_GROUP", "get_rank", "get_local_rank", "get_world_size", "is_primary", "synchronize",
    "gather", "data_sampler", "find_free_port", "launch", "job", "init_from_env", "all_reduce_mean",
    "broadcast_object", "device", "backend", "destroy",
]

LOCAL_PROCESS_GROUP = None
_LOCAL_RANK = 0
_DEFAULT_TIMEOUT = datetime.timedelta(minutes=int(os.environ.get("TBAMD_PG_TIMEOUT_MIN", "30")))


def _ready() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if _ready() else 0


def get_local_rank() -> int:
    if not _ready():
        return 0
    if LOCAL_PROCESS_GROUP is None:
        return _LOCAL_RANK
    return dist.get_rank(group=LOCAL_PROCESS_GROUP)


def get_world_size() -> int:
    return dist.get_world_size() if _ready() else 1


def is_primary() -> bool:
    return get_rank() == 0


def backend() -> Optional[str]:
    return dist.get_backend() if _ready() else None


def device() -> torch.device:
    """The device this rank computes on."""
    if torch.cuda.is_available() and backend() != "gloo":
        return torch.device("cuda", torch.cuda.current_device())
    if torch.cuda.is_available() and not _ready():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def synchronize() -> None:
    """Barrier across all ranks (no-op when not distributed)."""
    if not _ready() or dist.get_world_size() == 1:
        return
    if dist.get_backend() == "nccl":
        dist.barrier(device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier()


def gather(tensor: torch.Tensor, tensor_list: Optional[List[torch.Tensor]] = None) -> None:
    """Gather ``tensor`` from every rank into ``tensor_list`` on rank 0."""
    if not _ready():
        if tensor_list is not None and len(tensor_list) > 0:
            tensor_list[0].copy_(tensor)
        return
    if is_primary():
        dist.gather(tensor, tensor_list, dst=0)
    else:
        dist.gather(tensor, dst=0)


def all_reduce_mean(t: torch.Tensor) -> torch.Tensor:
    if _ready() and dist.get_world_size() > 1:
        dist.all_reduce(t)
        t /= dist.get_world_size()
    return t


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not _ready() or dist.get_world_size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def data_sampler(dataset: Dataset, shuffle: bool, distributed: bool) -> Sampler:
    if distributed and _ready():
        return DistributedSampler(dataset, shuffle=shuffle)
    if shuffle:
        return RandomSampler(dataset)
    return SequentialSampler(dataset)


def find_free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _make_local_groups(world_size: int, per_machine: int, machine_rank: int) -> None:
    global LOCAL_PROCESS_GROUP
    n_machine = max(1, world_size // max(1, per_machine))
    for i in range(n_machine):
        ranks = list(range(i * per_machine, (i + 1) * per_machine))
        g = dist.new_group(ranks)
        if i == machine_rank:
            LOCAL_PROCESS_GROUP = g


def _pick_backend(requested: Optional[str], use_cuda: bool) -> str:
    if requested:
        return requested.lower()
    # device_count() reads the device list without initialising the HIP runtime,
    # so a launching parent stays GPU-free (its children own the devices)
    return "nccl" if use_cuda and torch.cuda.device_count() > 0 else "gloo"


def _pg_options(be: str):
    """RCCL process-group options: the communicator's streams are created with
    HIGH priority, so a bucket all-reduce issued mid-backward is dispatched
    ahead of queued compute work instead of behind it."""
    if be != "nccl" or os.environ.get("TBAMD_RCCL_HIPRI", "1") == "0":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        # the same timeout as the init_process_group kwarg: torch overrides the options' value with
        # the kwarg and warns when the two differ (every RCCL init warned before round 4)
        opts._timeout = _DEFAULT_TIMEOUT
        return opts
    except Exception:  # pragma: no cover - backend built without NCCL/RCCL
        return None


def _streams_after_init() -> None:
    # the backward side stream must not share the compute stream's hardware queue under RCCL
    # (ops/streams.py _make_side, profiles/r06_ddp/queue_ab.txt)
    if dist.is_initialized() and dist.get_backend() == "nccl":
        from torchbooster_amd.ops import streams

        streams.on_process_group_init()


def init_from_env(backend: Optional[str] = None) -> bool:
    """Join a ``torchrun``-style launch (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_ADDR / MASTER_PORT in the environment).  Returns True if initialised."""
    global _LOCAL_RANK
    if _ready():
        return True
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        return False
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    use_cuda = (backend or "nccl") != "gloo"
    be = _pick_backend(backend, use_cuda)
    _LOCAL_RANK = local
    kw = {}
    if be == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
        kw["pg_options"] = _pg_options(be)
    dist.init_process_group(be, init_method="env://", world_size=world, rank=rank, timeout=_DEFAULT_TIMEOUT,
                            **kw)
    _streams_after_init()
    if world > 1:
        _make_local_groups(world, local_world, rank // max(1, local_world))
    return True


def destroy() -> None:
    global LOCAL_PROCESS_GROUP
    if _ready():
        try:
            dist.destroy_process_group()
        except Exception:  # pragma: no cover
            pass
    LOCAL_PROCESS_GROUP = None


def launch(fn: Callable, n_gpu_per_machine: int, n_machine: int = 1, machine_rank: int = 0,
           dist_url: Optional[str] = None, args: Tuple[Any, ...] = (), backend: Optional[str] = None,
           n_proc: int = 0) -> None:
    """Run ``fn(*args)`` on ``n_machine * n_gpu_per_machine`` ranks.

    * Under torchrun (env:// variables present) the current process joins and
      runs ``fn`` directly.
    * ``world_size == 1`` runs ``fn`` in-process without a process group (as the
      reference does).
    * ``n_gpu_per_machine == 0`` runs on CPU: in-process, or ``n_proc`` gloo
      ranks when ``n_proc > 1`` (A.2 B7: the reference silently ran nothing).
    * ``dist_url="auto"`` picks a free localhost port (single machine only).
    """
    from torchbooster_amd import utils as _utils

    if "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        init_from_env(backend)
        _utils._reapply_state(_utils._capture_state(), get_rank())
        fn(*args)
        return
    per_machine = n_gpu_per_machine
    use_cuda = n_gpu_per_machine > 0
    if n_gpu_per_machine == 0:
        per_machine = max(1, n_proc)
        backend = backend or "gloo"
    world_size = n_machine * per_machine
    if world_size == 1:
        fn(*args)
        return
    logging.info("Launching in distributed mode")
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    if dist_url in (None, "auto"):
        if n_machine > 1:
            raise ValueError("dist_url='auto' no supported in multi-machine jobs")
        dist_url = f"tcp://127.0.0.1:{find_free_port()}"
    state = _utils._capture_state()
    be = _pick_backend(backend, use_cuda)
    mp.spawn(job, nprocs=per_machine,
             args=(fn, world_size, per_machine, machine_rank, dist_url, args, be, state), daemon=False)


def job(local_rank: int, fn: Callable, world_size: int, n_gpu_per_machine: int, machine_rank: int = 0,
        dist_url: Optional[str] = None, args: Tuple[Any, ...] = (), backend: str = "nccl",
        state: Optional[dict] = None) -> None:
    """Body of one spawned rank (reference distributed.py:156-205)."""
    global LOCAL_PROCESS_GROUP, _LOCAL_RANK
    from torchbooster_amd import utils as _utils

    if backend == "nccl":
        if not torch.cuda.is_available():
            raise OSError("CUDA is not available on this machine")
        if n_gpu_per_machine > torch.cuda.device_count():
            raise ValueError(f"Asked for {n_gpu_per_machine} gpus but got {torch.cuda.device_count()} available")
        torch.cuda.set_device(local_rank)  # bind BEFORE any collective (B9)
    _LOCAL_RANK = local_rank
    global_rank = machine_rank * n_gpu_per_machine + local_rank
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", local_rank)
        kw["pg_options"] = _pg_options(backend)
    try:
        dist.init_process_group(backend=backend, init_method=dist_url, world_size=world_size, rank=global_rank,
                                timeout=_DEFAULT_TIMEOUT, **kw)
    except Exception as e:
        raise OSError(f"{backend.upper()} process group failed to initialize: {e}") from e
    _streams_after_init()
    if state is not None:
        _utils._reapply_state(state, global_rank)
    synchronize()
    if LOCAL_PROCESS_GROUP is not None:
        raise ValueError("torch.distributed.LOCAL_PROCESS_GROUP is not None")
    _make_local_groups(world_size, n_gpu_per_machine, machine_rank)
    try:
        fn(*args)
    except BaseException:
        # fail fast: no barrier / teardown collective here —
        # the peers may be blocked inside a different collective, so either
        # would hang; exiting lets mp.spawn terminate the remaining ranks
        raise
    synchronize()
    destroy()
