"""CycleScheduler curve parity (reference scheduler.py:70-172; SURVEY.md C14 verified trace)."""
import math

import pytest
import torch

from torchbooster_amd.scheduler import CycleScheduler, anneal_cos, anneal_exp, anneal_flat, anneal_linear


def opt(lr=1.0):
    return torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=lr)


def test_anneal_functions():
    assert anneal_linear(1, 3, 0.5) == 2
    assert anneal_cos(1, 0, 0) == pytest.approx(1) and anneal_cos(1, 0, 1) == pytest.approx(0)
    assert anneal_exp(1, 0.01, 0.5) == pytest.approx(0.1)
    assert anneal_flat(5, 0, 0.7) == 5


def test_reference_trace_warmup3_n10_lin_cos():
    o = opt(1.0)
    s = CycleScheduler(o, 1.0, 10, initial_multiplier=0.04, final_multiplier=0.0, warmup=3, decay=("lin", "cos"))
    lrs = [s.step() for _ in range(12)]
    # verified against the reference: .04,.36,.68,1.0 | 1.0,.9505,...,.0495,0.0 (each phase n+1 steps)
    assert lrs[:4] == pytest.approx([0.04, 0.36, 0.68, 1.0])
    anneal = [0.0 + 0.5 * (1.0 - 0.0) * (1 + math.cos(math.pi * t / 7)) for t in range(8)]
    assert lrs[4:12] == pytest.approx(anneal)
    assert lrs[5] == pytest.approx(0.9505, abs=1e-4) and lrs[10] == pytest.approx(0.0495, abs=1e-4)
    assert o.param_groups[0]["lr"] == lrs[-1]


def test_overrun_holds_final_lr():
    o = opt(1.0)
    s = CycleScheduler(o, 1.0, 4, final_multiplier=0.1, decay=("cos", "lin"))
    vals = [s.step() for _ in range(10)]  # reference raises IndexError (B3); we clamp
    assert vals[-1] == pytest.approx(0.1)


def test_plateau_phase_works():
    o = opt(2.0)
    s = CycleScheduler(o, 2.0, 10, warmup=2, plateau=3, decay=("lin", "lin"))
    assert [p[0] for p in s.phases] == ["lin", "lin", "lin"]  # B2: "linear" fixed
    vals = [s.step() for _ in range(7)]
    assert vals[3:7] == pytest.approx([2.0] * 4)


def test_state_dict_roundtrip_and_repr():
    o = opt()
    s = CycleScheduler(o, 1.0, 10, warmup=2)
    for _ in range(4):
        s.step()
    sd = s.state_dict()
    assert set(sd) == {"phases", "phase", "phase_step", "last_lr"}
    s2 = CycleScheduler(opt(), 1.0, 10, warmup=2)
    s2.load_state_dict(sd)
    assert s2.step() == s.step()
    assert repr(s) == "CycleScheduler(phases=['COS', 'COS'])"
