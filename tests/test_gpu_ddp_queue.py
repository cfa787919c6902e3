"""The backward side stream under an RCCL process group (ops/streams.py ``_make_side``, "auto").

With RCCL up, a normal-priority side stream from torch's pool shared the compute stream's hardware
queue. The weight gradients then ran in order behind the input-gradient chain: the 1-rank --ddp
bench lost 11.6 % (profiles/r06_ddp/queue_ab.txt). The auto rule makes the side stream low priority
whenever an RCCL group exists when the stream is created, and keeps the caller's priority otherwise.
Each case runs in a child process, because the side stream is created once per process.
Reference: the DDP step of /root/reference/torchbooster/distributed.py:110-205.
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import os, sys, torch
sys.path.insert(0, sys.argv[1])
import torch.distributed as tdist
from torchbooster_amd import distributed as dist
from torchbooster_amd.ops import streams
torch.cuda.set_device(0)
if sys.argv[2] == "rccl":
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(dist.find_free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    assert dist.init_from_env("nccl")
s = streams.side_stream(0)
print("PRIO", streams.SIDE_INFO[0][0], s.priority, torch.cuda.current_stream().priority)
if tdist.is_initialized():
    tdist.destroy_process_group()
"""


def _child(mode: str):
    env = dict(os.environ)
    env.pop("TBAMD_SIDE_PRIORITY", None)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, mode], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("PRIO")][-1]
    return [int(v) for v in line.split()[1:]]


def test_side_stream_below_compute_under_rccl():
    used, side, compute = _child("rccl")
    assert used > 0 and side == used, (used, side, compute)  # HIP's least priority: its own queue class
    assert side > compute


def test_side_stream_at_callers_priority_without_a_group():
    used, side, compute = _child("plain")
    assert used == 0 and side == compute, (used, side, compute)


_CHILD_LATE = r"""
import os, sys, torch
sys.path.insert(0, sys.argv[1])
from torchbooster_amd import distributed as dist
from torchbooster_amd.ops import streams
torch.cuda.set_device(0)
before = streams.side_stream(0)  # made before the group, at the caller's priority
torch.cuda.synchronize()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(dist.find_free_port()), RANK="0", WORLD_SIZE="1",
                  LOCAL_RANK="0")
assert dist.init_from_env("nccl")
after = streams.side_stream(0)
print("PRIO", before.priority, after.priority, int(after.cuda_stream != before.cuda_stream))
dist.destroy()
"""


def test_side_stream_made_before_the_group_is_replaced():
    env = dict(os.environ)
    env.pop("TBAMD_SIDE_PRIORITY", None)
    r = subprocess.run([sys.executable, "-c", _CHILD_LATE, ROOT], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    before, after, replaced = [int(v) for v in [x for x in r.stdout.splitlines() if x.startswith("PRIO")][-1].split()[1:]]
    assert replaced == 1 and after > before, (before, after, replaced)
