"""utils.GraphedStep: a whole training step captured once and replayed (hipGraph).

CPU: the wrapper runs the step eagerly (same results as a plain loop).  GPU:
graph replays must reproduce the eager trajectory, schedulers included."""
import copy

import pytest
import torch
import torch.nn.functional as F

from torchbooster_amd import utils
from torchbooster_amd.scheduler import CycleScheduler


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(), torch.nn.Linear(64, 10))


def _run(model, opt, sched, batches, graphed, warmup=2):
    def train(x, y):
        loss = F.cross_entropy(model(x).float(), y)
        utils.step(loss, opt, clip=1.0)
        return loss.detach()

    fn = utils.GraphedStep(train, [opt], [sched], warmup=warmup) if graphed else None
    losses = []
    for x, y in batches:
        if graphed:
            losses.append(fn(x, y).clone())
        else:
            losses.append(train(x, y))
            sched.step()
    return torch.stack(losses)


def _batches(dev, n=7, dtype=torch.float32):
    g = torch.Generator().manual_seed(1)
    return [(torch.randn(16, 32, generator=g).to(dev, dtype), torch.randint(0, 10, (16,), generator=g).to(dev))
            for _ in range(n)]


def test_graph_step_cpu_eager_equivalence():
    from torchbooster_amd.ops.optim import FusedAdamW

    a = _mlp()
    b = copy.deepcopy(a)
    oa, ob = FusedAdamW(a.parameters(), lr=1e-2), FusedAdamW(b.parameters(), lr=1e-2)
    sa, sb = CycleScheduler(oa, 1e-2, 20, warmup=3), CycleScheduler(ob, 1e-2, 20, warmup=3)
    la = _run(a, oa, sa, _batches("cpu"), False)
    lb = _run(b, ob, sb, _batches("cpu"), True)
    assert torch.allclose(la, lb)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p, q)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("opt_name", ["adamw", "sgd"])
def test_graph_step_gpu_matches_eager(opt_name):
    from torchbooster_amd.ops.linear import Linear, LinearGELU
    from torchbooster_amd.ops.optim import FusedAdamW, FusedSGD

    torch.manual_seed(0)
    a = torch.nn.Sequential(LinearGELU(32, 64), Linear(64, 10)).cuda()
    b = copy.deepcopy(a)

    def mk(m):
        if opt_name == "adamw":
            o = FusedAdamW(m.parameters(), lr=1e-2)
        else:
            o = FusedSGD(m.parameters(), lr=1e-2, momentum=0.9)
        return o, CycleScheduler(o, 1e-2, 20, warmup=3)

    oa, sa = mk(a)
    ob, sb = mk(b)
    la = _run(a, oa, sa, _batches("cuda"), False)
    lb = _run(b, ob, sb, _batches("cuda"), True)
    torch.cuda.synchronize()
    assert torch.allclose(la, lb, rtol=1e-5, atol=1e-6), (la, lb)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6)
    assert oa.param_groups[0]["step"] == ob.param_groups[0]["step"] == 7
    assert abs(oa.param_groups[0]["lr"] - ob.param_groups[0]["lr"]) < 1e-12


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_graph_step_pixel_optimisation_with_hooks():
    """NST-style step (examples/img_stt/offline): frozen conv net, forward hooks that keep
    the previous step's features alive, the image is the only parameter."""
    from torchbooster_amd.ops.conv import Conv2d
    from torchbooster_amd.ops.optim import FusedAdamW

    torch.manual_seed(0)
    net = torch.nn.Sequential(Conv2d(3, 64, 3, 1, 1), torch.nn.ReLU(), Conv2d(64, 64, 3, 1, 1), torch.nn.ReLU(),
                              Conv2d(64, 128, 3, 1, 1)).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    for p in net.parameters():
        p.requires_grad_(False)
    feats = {}
    for i in (0, 4):
        net[i].register_forward_hook(lambda m, a, o, i=i: feats.__setitem__(i, o))
    target = torch.randn(1, 128, 32, 32, device="cuda")

    def run(graphed):
        img = torch.rand(1, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
        img.requires_grad_(True)
        opt = FusedAdamW([img], lr=0.05, weight_decay=0.0)

        def train():
            net(img.to(torch.bfloat16))
            loss = (feats[4].float() - target).pow(2).mean() + feats[0].float().abs().mean()
            utils.step(loss, opt)
            return loss.detach()

        fn = utils.GraphedStep(train, [opt], [], warmup=2) if graphed else train
        return torch.stack([fn().clone() for _ in range(6)]), img.detach()

    torch.manual_seed(3)
    la, ia = run(False)
    torch.manual_seed(3)
    lb, ib = run(True)
    torch.cuda.synchronize()
    assert torch.isfinite(lb).all()
    assert torch.allclose(la, lb, rtol=1e-3, atol=1e-4), (la, lb)
    assert torch.allclose(ia, ib, rtol=1e-3, atol=1e-3)
