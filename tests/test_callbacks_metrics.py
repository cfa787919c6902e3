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
    assert set(ck) == {"model", "optim", "scheduler", "epoch"}
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
