"""Rank-0-authoritative routing decisions (ops/_agree.py): on a gloo world of 3 every rank
takes rank 0's published decision, and a key rank 0 never publishes times out to the local one."""
import os

import pytest
import torch.multiprocessing as mp

from torchbooster_amd import distributed as dist


def _worker(rank, world, port, q):
    os.environ["TBAMD_TUNE_AGREE_TIMEOUT"] = "2"
    import importlib

    import torch.distributed as tdist

    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from torchbooster_amd.ops import _agree

    importlib.reload(_agree)
    key = ("fwd", (256, 64, 56, 56), (64, 64, 3, 3), 1, 1)
    if rank == 0:
        assert _agree.shared("conv", key) is None
        _agree.publish("conv", key, "native")
        _agree.publish("gemm", ("nt", 100, 64, 32), [16, 1])
    got = _agree.shared("conv", key)
    gemm = _agree.shared("gemm", ("nt", 100, 64, 32))
    missing = _agree.shared("conv", ("never", rank))
    # a slow first-use timing on rank 0 (longer than the start timeout): the other ranks saw the
    # started mark and wait for the decision instead of deciding for themselves
    slow = ("fwd", "slow")
    if rank == 0:
        assert _agree.shared("conv", slow) is None
        import time

        time.sleep(3.0)
        _agree.publish("conv", slow, "miopen")
    got_slow = _agree.shared("conv", slow)
    tdist.barrier()
    q.put((rank, got, gemm, missing, got_slow, len(_agree.FALLBACKS)))
    tdist.destroy_process_group()


@pytest.mark.timeout(120)
def test_rank0_decision_is_shared():
    world = 3
    port = dist.find_free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert res[0] == (0, None, None, None, None, 0)
    for r in (1, 2):
        assert res[r] == (r, "native", [16, 1], None, "miopen", 1)  # one logged fallback: ("never", r)
