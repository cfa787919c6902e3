"""utils.* behaviour (reference utils.py) including the A.2 fixes."""
from collections import namedtuple

import pytest
import torch

from torchbooster_amd import utils


def test_step_order_and_clip():
    torch.manual_seed(0)
    m = torch.nn.Linear(4, 1)
    o = torch.optim.SGD(m.parameters(), lr=0.1)
    x = torch.randn(8, 4)
    w0 = m.weight.detach().clone()
    loss = (m(x) ** 2).mean() * 1000
    utils.step(loss, o, clip=1.0)
    # clipped to unit norm => the update's norm is at most lr
    upd = torch.cat([(m.weight - w0).flatten()])
    assert upd.norm() <= 0.1 + 1e-6


def test_step_accumulate_keeps_grads():  # B6
    p = torch.nn.Parameter(torch.zeros(1))
    o = torch.optim.SGD([p], lr=1.0)
    utils.step((p * 1.0).sum(), o, accumulate=True)
    utils.step((p * 2.0).sum(), o)
    assert p.item() == pytest.approx(-3.0)  # reference would give -2 (grads wiped)
    utils.step((p * 1.0).sum(), o)
    assert p.item() == pytest.approx(-4.0)


def test_seed_deterministic_kwarg():  # B5
    utils.seed(3, deterministic=False)
    a = torch.rand(3)
    utils.seed(3, deterministic=True)
    b = torch.rand(3)
    assert torch.equal(a, b)
    torch.use_deterministic_algorithms(False)


def test_freeze_detach():
    m = torch.nn.Linear(2, 2)
    utils.freeze(m)
    assert not any(p.requires_grad for p in m.parameters())
    a = torch.ones(2, requires_grad=True)
    assert not utils.detach(a * 2).requires_grad
    x, y = utils.detach(a * 2, a * 3)
    assert not x.requires_grad and not y.requires_grad


def test_iter_loader_epochs_and_set_epoch():
    class S(torch.utils.data.Sampler):
        def __init__(self):
            self.epochs = []

        def set_epoch(self, e):
            self.epochs.append(e)

        def __iter__(self):
            return iter(range(3))

        def __len__(self):
            return 3

    s = S()
    dl = torch.utils.data.DataLoader(list(range(3)), batch_size=2, sampler=s)
    it = utils.iter_loader(dl)
    got = [next(it)[0] for _ in range(5)]
    assert got == [0, 0, 1, 1, 2]
    assert s.epochs[:3] == [0, 1, 2]


def test_to_tensor_and_stack():
    assert utils.to_tensor([1, 2], dtype=torch.float64).dtype == torch.float64  # B17
    P = namedtuple("P", "a b")
    t = utils.to_tensor(P(1, [2, 3]))
    assert isinstance(t, P) and t.b.shape == (2,)
    d = utils.to_tensor({"x": [1.0]})
    assert d["x"].shape == (1,)
    st = utils.stack_dictionaries([{"a": torch.ones(2)}, {"a": torch.zeros(2)}])
    assert st["a"].shape == (2, 2)
    assert utils.stack_dictionaries([]) == {}
    assert utils.isinstance_namedtuple(P(1, 2)) and not utils.isinstance_namedtuple((1, 2))


def test_step_with_scaler_and_scheduler():
    from torchbooster_amd.scheduler import CycleScheduler

    m = torch.nn.Linear(2, 1)
    o = torch.optim.AdamW(m.parameters(), lr=1e-2)
    s = CycleScheduler(o, 1e-2, 10, warmup=2)
    scaler = torch.amp.GradScaler("cpu", enabled=True)
    loss = m(torch.ones(3, 2)).sum()
    utils.step(loss, o, scheduler=s, scaler=scaler, clip=1.0)
    assert s.last_lr is not None
