"""The native reducer on RCCL (backend "nccl" on ROCm) on the GPU.

A 1-rank RCCL group with ``force_reduce=True`` runs the whole reducer path on
hardware -- post-accumulate hooks, in-order bucket release, grouped mixed-dtype
collectives on the high-priority communicator stream, finalize -- and must give
parameters bit-identical to the unwrapped native model after 3 AdamW steps (an
AVG all-reduce over one rank is exact).  Multi-rank equality is covered on gloo
(tests/test_distributed.py); the driver's 8-GPU bench runs the same code.

Reference: DDP wrap in to_env (/root/reference/torchbooster/config.py:176-178).
"""
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import torch.distributed as tdist  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
from torchbooster_amd import models, utils  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402
from torchbooster_amd.parallel import DistributedDataParallel  # noqa: E402


@pytest.fixture
def rccl_group(monkeypatch):
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(dist.find_free_port()))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert dist.init_from_env("nccl")
    assert tdist.get_backend() == "nccl"
    yield
    dist.destroy()


def _train(model, opt, x, y, steps=3):
    for _ in range(steps):
        loss, _ = cross_entropy_accuracy(model(x), y, 0.1)
        utils.step(loss, opt, clip=1.0)
    torch.cuda.synchronize()


def test_rccl_reducer_matches_unwrapped(rccl_group):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    base = models.resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    plain = copy.deepcopy(base)
    plain2 = copy.deepcopy(base)
    wrapped_inner = copy.deepcopy(base)
    ddp = DistributedDataParallel(wrapped_inner, force_reduce=True, bucket_cap_mb=4.0)
    launched = []
    orig = ddp._launch
    ddp._launch = lambda b: (launched.append(b), orig(b))[1]

    # xGMI bucket plan: contiguous mixed-dtype buckets, none below the 1 MiB floor but the last
    sizes = ddp.bucket_sizes_mb()
    assert len(sizes) > 2
    assert all(s >= 1.0 for s in sizes[:-1]), sizes
    kinds = [sorted({d for d, _ in parts}) for parts in ddp.bucket_layout()]
    assert any(k == ["bfloat16", "float32"] for k in kinds), kinds  # BN f32 params ride with their convs

    x = torch.randn(16, 3, 64, 64, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=dev)
    o1 = FusedAdamW(plain.parameters(), lr=1e-3, weight_decay=1e-2)
    o2 = FusedAdamW(ddp.parameters(), lr=1e-3, weight_decay=1e-2)
    o3 = FusedAdamW(plain2.parameters(), lr=1e-3, weight_decay=1e-2)
    # deterministic mode (what utils.seed() sets): native fixed-order kernels only, so an AVG
    # all-reduce over ONE rank must leave every gradient and every parameter bit-identical
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        _train(plain2, o3, x, y, steps=1)  # (route autotuning of the deterministic candidates)
        loss, _ = cross_entropy_accuracy(plain(x), y, 0.1)
        o1.zero_grad(set_to_none=True)
        loss.backward()
        g_plain = {n: p.grad.detach().clone() for n, p in plain.named_parameters()}
        loss, _ = cross_entropy_accuracy(ddp(x), y, 0.1)
        o2.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        for n, p in wrapped_inner.named_parameters():
            assert torch.equal(p.grad, g_plain[n]), (n, (p.grad.float() - g_plain[n].float()).abs().max().item())
        o1.step()
        o2.step()
        _train(plain, o1, x, y, steps=2)
        _train(ddp, o2, x, y, steps=2)
    finally:
        torch.use_deterministic_algorithms(prev)
    assert sorted(set(launched)) == list(range(ddp.num_buckets))  # every bucket went through RCCL
    assert len(launched) == 3 * ddp.num_buckets
    for (n, a), b in zip(plain.named_parameters(), wrapped_inner.parameters()):
        assert torch.equal(a, b), (n, (a.float() - b.float()).abs().max().item())


def test_rccl_pg_uses_high_priority_streams(rccl_group):
    pg = tdist.distributed_c10d._get_default_group()
    opts = getattr(pg._get_backend(torch.device("cuda", 0)), "options", None)
    if opts is None:  # pragma: no cover - older torch
        pytest.skip("backend options not exposed")
    assert opts.is_high_priority_stream
    assert os.environ.get("TBAMD_RCCL_HIPRI", "1") != "0"


def test_rccl_effective_timeout_and_no_override_warning(monkeypatch):
    """The communicator runs with the job's PG timeout (TBAMD_PG_TIMEOUT_MIN) and init raises no
    'backend_options._timeout ... will always override it' warning."""
    import warnings

    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(dist.find_free_port()))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert dist.init_from_env("nccl")
    try:
        assert not [x for x in w if "_timeout" in str(x.message)], [str(x.message) for x in w]
        pg = tdist.distributed_c10d._get_default_group()
        opts = pg._get_backend(torch.device("cuda", 0)).options
        assert opts._timeout == dist._DEFAULT_TIMEOUT
    finally:
        dist.destroy()


def test_rccl_reducer_with_bn_in_operand_bottlenecks(rccl_group, monkeypatch):
    """ResNet-50 at a size where the default BN-in-operand path (bn2 -> persistent conv3, weight
    gradient on the side stream into the reducer's slots) engages: one backward through the 1-rank
    RCCL reducer gives gradients bit-identical to the unwrapped model (deterministic mode)."""
    from torchbooster_amd.models import resnet as RN

    calls = [0]
    orig = RN.conv2d_xf_bn_stats

    def counted(*a, **k):
        calls[0] += 1
        return orig(*a, **k)

    monkeypatch.setattr(RN, "conv2d_xf_bn_stats", counted)
    monkeypatch.setattr(RN, "_LAZY_BN", True)
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    base = models.resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    plain = copy.deepcopy(base)
    wrapped_inner = copy.deepcopy(base)
    ddp = DistributedDataParallel(wrapped_inner, force_reduce=True)
    x = torch.randn(48, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (48,), device=dev)
    o1 = FusedAdamW(plain.parameters(), lr=1e-3, weight_decay=1e-2)
    o2 = FusedAdamW(ddp.parameters(), lr=1e-3, weight_decay=1e-2)
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        warm = copy.deepcopy(base)
        _train(warm, FusedAdamW(warm.parameters(), lr=1e-3), x, y, steps=1)  # route tuning
        calls[0] = 0
        loss, _ = cross_entropy_accuracy(plain(x), y, 0.1)
        o1.zero_grad(set_to_none=True)
        loss.backward()
        g_plain = {n: p.grad.detach().clone() for n, p in plain.named_parameters()}
        loss, _ = cross_entropy_accuracy(ddp(x), y, 0.1)
        o2.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        assert calls[0] == 2 * 7, calls[0]  # stage 1-2 bottlenecks, both models
        for n, p in wrapped_inner.named_parameters():
            assert torch.equal(p.grad, g_plain[n]), (n, (p.grad.float() - g_plain[n].float()).abs().max().item())
    finally:
        torch.use_deterministic_algorithms(prev)
