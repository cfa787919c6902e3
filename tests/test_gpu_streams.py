"""Backward side stream for conv weight gradients (ops/streams.py): gradients, and the
parameters after a few FusedAdamW steps, match with the split on and off, and
the side stream was used.""" 
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.ops import streams  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402


def _run(split: bool, steps: int = 3):
    streams.set_enabled(split)
    try:
        torch.manual_seed(0)
        m = models.resnet18(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        opt = FusedAdamW(m.parameters(), lr=1e-3)
        g = torch.Generator(device="cuda").manual_seed(1)
        grads = []
        for _ in range(steps):
            x = torch.randn(16, 3, 64, 64, device="cuda", generator=g).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 10, (16,), device="cuda", generator=g)
            opt.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(m(x).float(), y).backward()
            assert not any(streams._PENDING.values())  # joined when backward() returned
            grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
            opt.step()
        return grads, {n: p.detach().clone() for n, p in m.named_parameters()}
    finally:
        streams.set_enabled(True)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _worst(a, b):
    return max((_rel(a[n], b[n]), n) for n in a)


@pytest.fixture
def deterministic():
    """Deterministic mode (what utils.seed() sets): the conv / GEMM routers keep to the native
    fixed-order kernels -- MIOpen's split-K solvers (float atomics) won the few-pixel layer-4
    shapes of this model and made two identical runs differ by a bf16 ulp in a few outputs,
    which the optimizer then amplified (scripts/r4/nondet_fwd.py)."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    yield
    torch.use_deterministic_algorithms(prev)


def test_side_stream_wgrad_matches_single_stream(deterministic):
    """Gradients and updated parameters with the split on are BITWISE those of the
    single-stream run (every kernel is fixed-order in deterministic mode)."""
    _run(False)  # first use of every shape: route autotuning
    g0, p0 = _run(False)
    g0b, p0b = _run(False)
    g1, p1 = _run(True)
    assert streams._SIDE, "the side stream was never used"
    for step in range(len(g0)):
        assert _worst(g0b[step], g0[step])[0] == 0.0, (step, _worst(g0b[step], g0[step]))
        assert _worst(g1[step], g0[step])[0] == 0.0, (step, _worst(g1[step], g0[step]))
    assert _worst(p1, p0)[0] == 0.0


def test_stop_event_fork_matches_marker_fork(deterministic):
    """The fork that waits on the BN backward kernel's own completion event (ops/streams.py
    arm / tag) gives the same gradients as the marker fork, and is the one taken."""
    _run(True)  # warm-up: route autotuning
    streams._STOP_EVENTS = False
    try:
        g0, p0 = _run(True)
    finally:
        streams._STOP_EVENTS = True
    before = dict(streams.FORKS)
    g1, p1 = _run(True)
    g1b, p1b = _run(True)
    took = streams.FORKS["stop_event"] - before["stop_event"]
    assert took > 0, streams.FORKS
    for step in range(len(g0)):
        assert _worst(g1[step], g0[step])[0] == 0.0, (step, _worst(g1[step], g0[step]))
    assert _worst(p1, p0)[0] == 0.0


def test_side_stream_with_a_fresh_tensor_wgrad_route():
    """A weight-gradient route that returns a fresh tensor (MIOpen) instead of writing the slot
    lands it in the slot on the side stream: gradients match the single-stream run."""
    from torchbooster_amd.ops import conv as CV

    old = CV._FORCE["wgrad"]
    CV._FORCE["wgrad"] = "miopen"
    try:
        _run(False)
        g0, p0 = _run(False)
        g0b, _ = _run(False)
        g1, p1 = _run(True)
    finally:
        CV._FORCE["wgrad"] = old
    for step in range(len(g0)):
        base = _worst(g0b[step], g0[step])[0]
        got = _worst(g1[step], g0[step])
        assert got[0] <= max(4 * base, 2e-3), (step, got, base)


def test_step_keeps_the_callers_stream():
    """``utils.step`` (and ``EnvironementConfig.make``) never change the
    process's current stream (the side-stream weight gradients run on their own stream: at the
    caller's priority by default, at the lowest HIP priority with TBAMD_SIDE_PRIORITY=low)."""
    from torchbooster_amd import utils
    from torchbooster_amd.config import EnvironementConfig

    before = torch.cuda.current_stream().cuda_stream
    m = models.resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    x = torch.randn(8, 3, 64, 64, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    utils.step(m(x).float().square().mean(), opt)
    assert torch.cuda.current_stream().cuda_stream == before
    EnvironementConfig(n_gpu=1).make(torch.nn.Linear(4, 4))
    assert torch.cuda.current_stream().cuda_stream == before
    if streams.enabled() and streams._SIDE_PRIORITY == "low":
        prio, least, greatest = streams.SIDE_INFO[torch.cuda.current_device()]
        print("side stream priority", prio, "range", least, greatest)
        if least is not None and least > 0:
            side = streams.side_stream(torch.cuda.current_device())
            assert side.priority == least  # the least (numerically largest) priority


def test_step_in_user_stream_context_orders_correctly():
    """A training loop inside its own ``torch.cuda.stream`` context: the step joins that stream
    (priority stream waits for it), the stream is unchanged afterwards, and work queued on it
    after the step sees the updated parameters (the user stream waits for the step)."""
    from torchbooster_amd import utils

    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 256).cuda()
    ref = torch.nn.Linear(256, 256).cuda()
    ref.load_state_dict(lin.state_dict())
    opt = FusedAdamW(lin.parameters(), lr=1e-2, weight_decay=0.0)
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    x = torch.randn(512, 256, device="cuda")
    us = torch.cuda.Stream()
    us.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(us):
        for _ in range(3):
            # a long user-stream producer right before the loss: the step must wait for it
            xx = (x @ torch.eye(256, device="cuda")).relu()
            utils.step(lin(xx).square().mean(), opt)
            assert torch.cuda.current_stream().cuda_stream == us.cuda_stream
            w_after = lin.weight.clone()  # queued on us right after the step
    torch.cuda.synchronize()
    for _ in range(3):
        ropt.zero_grad()
        ref(x.relu()).square().mean().backward()
        ropt.step()
    torch.testing.assert_close(w_after, ref.weight.detach(), rtol=1e-4, atol=1e-5)


