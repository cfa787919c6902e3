"""SaveCallback layout (reference callbacks.py:75-129) and metrics (metrics.py)."""
import torch

from torchbooster_amd.callbacks import BaseCallback, SaveCallback, load_checkpoint, try_extract_state_dict
from torchbooster_amd.metrics import Accuracy, RunningAverage, accuracy
from torchbooster_amd.scheduler import CycleScheduler


def test_save_callback_names_and_content(tmp_path):
    m = torch.nn.Linear(2, 2)
    o = torch.optim.AdamW(m.parameters())
    s = CycleScheduler(o, 1e-3, 10)
    cb = SaveCallback(every=3, n_iter=100, root=tmp_path, prefix="run")
    for e in range(7):
        cb(model=m, optim=o, scheduler=s, epoch=e)
    names = sorted(f.name for f in tmp_path.iterdir())
    assert names == ["run_003.pt", "run_006.pt"]
    ck = torch.load(tmp_path / "run_006.pt", weights_only=True)
    assert set(ck) == {"model", "optim", "scheduler", "epoch"}  # the reference's keys, nothing added
    assert set(ck["model"]) == {"weight", "bias"}  # no "module." prefix
    assert ck["epoch"] == 5
    assert ck["scheduler"]["phase"] == 0


def test_ddp_like_unwrap_and_scaler():
    m = torch.nn.Linear(2, 2)

    class Wrap(torch.nn.Module):
        def __init__(self, mod):
            super().__init__()
            self.module = mod

    sd = try_extract_state_dict(Wrap(m))
    assert set(sd) == {"weight", "bias"}
    scaler = torch.amp.GradScaler("cpu", enabled=True)
    assert isinstance(try_extract_state_dict(scaler), dict)  # B15
    assert try_extract_state_dict(5) == 5


def test_resume(tmp_path):
    m = torch.nn.Linear(2, 2)
    cb = SaveCallback(every=2, n_iter=10, root=tmp_path, prefix="ck")
    for _ in range(4):
        cb(model=m)
    m2 = torch.nn.Linear(2, 2)
    cb2 = SaveCallback(every=2, n_iter=10, root=tmp_path, prefix="ck")
    cb2.resume(model=m2)
    assert cb2.current == 4
    assert torch.equal(m2.weight, m.weight)
    out = load_checkpoint(tmp_path / "ck_04.pt", model=torch.nn.Linear(2, 2))
    assert "model" in out


def test_base_callback_counts():
    class C(BaseCallback):
        def update(self, *a, **k):
            self.last = self.current

    c = C()
    c()
    c()
    assert c.current == 2 and c.last == 2


def test_accuracy_and_running_average():
    logits = torch.tensor([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7], [0.6, 0.4]])
    labels = torch.tensor([1, 0, 0, 0])
    assert accuracy(logits, labels).item() == 0.75
    assert Accuracy()(logits, labels).item() == 0.75
    ra = RunningAverage()
    for v in [1.0, 2.0, 3.0]:
        ra.update(v)
    assert ra.value == 2.0 and ra.current == 3
    rt = RunningAverage()
    for v in [1.0, 2.0, 3.0, 6.0]:
        rt.update(torch.tensor(v))
    assert abs(rt.value - 3.0) < 1e-6


def test_exact_resume_restores_rng_and_sampler_epoch(tmp_path):
    """a resumed run continues the same random streams (Python /
    NumPy / torch) and the same DistributedSampler epoch as an uninterrupted one."""
    import random

    import numpy as np
    from torch.utils.data import DataLoader, DistributedSampler

    ds = list(range(32))
    sampler = DistributedSampler(ds, num_replicas=2, rank=0, shuffle=True, seed=7)
    loader = DataLoader(ds, batch_size=4, sampler=sampler)
    sampler.set_epoch(5)
    model = torch.nn.Linear(3, 2)
    cb = SaveCallback(1, 10, tmp_path, "run", save_rng=True)  # exact-resume RNG state is opt-in
    random.seed(1), np.random.seed(2), torch.manual_seed(3)
    cb(model=model, loader=loader)
    want = (random.random(), float(np.random.rand()), float(torch.rand(1)), list(iter(sampler)))
    # clobber every stream and the epoch, then resume
    random.seed(99), np.random.seed(99), torch.manual_seed(99)
    sampler.set_epoch(0)
    cb2 = SaveCallback(1, 10, tmp_path, "run")
    ck = cb2.resume(model=model, loader=loader)
    assert cb2.current == 1 and ck["loader"] == {"sampler_epoch": 5}
    got = (random.random(), float(np.random.rand()), float(torch.rand(1)), list(iter(sampler)))
    assert got == want


def test_optimizer_config_ema():
    from torchbooster_amd.config import OptimizerConfig
    from torchbooster_amd.ops.optim import FusedAdamW

    m = torch.nn.Linear(4, 4)
    opt = OptimizerConfig(name="adamw", lr=1e-2, ema=0.5).make(m.parameters())
    assert isinstance(opt, FusedAdamW) and opt.ema_decay == 0.5
    w0 = m.weight.detach().clone()
    m(torch.randn(8, 4)).square().mean().backward()
    opt.step()
    ema = opt.ema_tensor(m.weight)
    # ema = 0.5 * w0 + 0.5 * w1 after the first step (EMA initialised from the weights)
    assert torch.allclose(ema, 0.5 * w0 + 0.5 * m.weight.detach(), atol=1e-6)
    import pytest

    with pytest.raises(ValueError):
        OptimizerConfig(name="sgd", lr=1e-2, ema=0.5).make(m.parameters())
