"""A conv weight used by several nodes of ONE backward.

The DCGAN discriminator runs on real and fake batches before one backward (ref GAN loop:
/root/reference/examples/img_gen/gan/gan.py:102-113), a weight-tied block repeats one module
(ref online.py:52-57): the first conv backward takes the parameter's zero-copy gradient slot
and writes it on the backward side stream (ops/streams.py); later ones return fresh tensors
that autograd sums with the slot alias on the compute stream.  That sum (and the DDP bind copy
of it into the slot) must wait for the side stream: gradients with the split on must equal
the single-stream ones, with and without the native reducer.
"""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import torch.distributed as tdist  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
from torchbooster_amd.ops import streams  # noqa: E402
from torchbooster_amd.ops.conv import Conv2d  # noqa: E402
from torchbooster_amd.ops.norm import BatchNormAct2d  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402
from torchbooster_amd.parallel import DistributedDataParallel  # noqa: E402


class _D(nn.Module):
    def __init__(self):
        super().__init__()
        self.c1 = Conv2d(64, 128, 3, 1, 1, bias=False)
        self.b1 = BatchNormAct2d(128, act="relu")
        self.c2 = Conv2d(128, 128, 3, 1, 1, bias=False)  # applied twice per forward (weight tying)
        self.b2 = BatchNormAct2d(128, act="relu")
        self.head = Conv2d(128, 64, 1, 1, 0, bias=False)

    def forward(self, x):
        h = self.b1(self.c1(x))
        h = self.b2(self.c2(h))
        h = self.c2(h)
        return self.head(h).float().mean(dim=(1, 2, 3))


def _grads(split: bool, ddp: bool, steps: int = 2):
    streams.set_enabled(split)
    try:
        torch.manual_seed(0)
        d = _D().cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        net = DistributedDataParallel(d, force_reduce=True, bucket_cap_mb=1.0) if ddp else d
        opt = FusedAdamW(net.parameters(), lr=1e-3)
        g = torch.Generator(device="cuda").manual_seed(1)
        out = []
        for _ in range(steps):
            real = torch.randn(8, 64, 32, 32, device="cuda", generator=g).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            fake = torch.randn(8, 64, 32, 32, device="cuda", generator=g).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            opt.zero_grad(set_to_none=True)
            # D(real) and D(fake) in one backward: every weight gets two contributions
            loss = torch.relu(1 - net(real)).mean() + torch.relu(1 + net(fake)).mean()
            loss.backward()
            torch.cuda.synchronize()
            out.append({n: p.grad.detach().clone() for n, p in d.named_parameters()})
            opt.step()
        return out
    finally:
        streams.set_enabled(True)


@pytest.fixture
def rccl_group(monkeypatch):
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(dist.find_free_port()))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert dist.init_from_env("nccl")
    yield
    dist.destroy()


def _check(a, b):
    for step, (ga, gb) in enumerate(zip(a, b)):
        for n in ga:
            assert torch.equal(ga[n], gb[n]), (step, n, (ga[n].float() - gb[n].float()).abs().max().item())


@pytest.fixture(autouse=True)
def deterministic():
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)  # native fixed-order kernels only
    yield
    torch.use_deterministic_algorithms(prev)


def test_shared_conv_weight_side_stream():
    _grads(False, False)  # first use of the shapes: route autotuning
    ref = _grads(False, False)
    got = _grads(True, False)
    assert streams._SIDE, "the side stream was never used"
    _check(got, ref)


def test_shared_conv_weight_side_stream_reducer(rccl_group):
    assert tdist.get_backend() == "nccl"
    _grads(False, True)
    ref = _grads(False, True)
    got = _grads(True, True)
    _check(got, ref)
