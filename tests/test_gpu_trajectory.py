"""20-step training trajectories on the native kernels against stock PyTorch (VERDICT r2
item 8): ResNet-18 (torchvision layout, nativized) at CIFAR shape, batch 256, and ViT-tiny.

Three runs from one initialisation over the same fixed batches:

* fp32 stock   -- the truth (ATen, fp32 weights, ``torch.optim.AdamW``);
* bf16 stock   -- ATen under ``torch.autocast(bfloat16)`` with fp32 master weights: the
                  error budget a user of stock mixed precision already accepts;
* bf16 native  -- nativized / native model in bf16, channels-last, ``FusedAdamW`` with
                  fp32 master weights.

The native loss curve must stay as close to the fp32 curve as the stock bf16 one does
(1.5x its mean deviation + 0.02) and must go down."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.nativize import nativize  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

STEPS = 20


def _batches(n, B, img, classes, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [(torch.randn(B, 3, img, img, device="cuda", generator=g),
             torch.randint(0, classes, (B,), device="cuda", generator=g)) for _ in range(n)]


def _train(model, data, opt, *, dtype=None, autocast=False):
    losses = []
    for i in range(STEPS):
        x, y = data[i % len(data)]
        x = x.contiguous(memory_format=torch.channels_last)
        if dtype is not None:
            x = x.to(dtype)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            out = model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return torch.tensor(losses)


def _check(l32, lamp, lnat):
    dev_amp = (lamp - l32).abs().mean().item()
    dev_nat = (lnat - l32).abs().mean().item()
    assert torch.isfinite(lnat).all()
    assert dev_nat <= 1.5 * dev_amp + 0.02, (dev_nat, dev_amp, lnat.tolist(), l32.tolist())
    assert lnat[-3:].mean() < lnat[:3].mean(), lnat.tolist()


def test_resnet18_cifar_b256_trajectory():
    torch.manual_seed(0)
    base = models.tv.resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    data = _batches(4, 256, 32, 10, seed=1)

    m32 = copy.deepcopy(base)
    l32 = _train(m32, data, torch.optim.AdamW(m32.parameters(), lr=1e-3))
    mamp = copy.deepcopy(base)
    lamp = _train(mamp, data, torch.optim.AdamW(mamp.parameters(), lr=1e-3), autocast=True)
    mnat = nativize(copy.deepcopy(base).to(torch.bfloat16))
    lnat = _train(mnat, data, FusedAdamW(mnat.parameters(), lr=1e-3), dtype=torch.bfloat16)
    _check(l32, lamp, lnat)


def test_vit_tiny_trajectory(monkeypatch):
    torch.manual_seed(0)
    base = models.vit.vit_tiny(num_classes=10, image=32).cuda()
    data = _batches(4, 128, 32, 10, seed=2)
    with monkeypatch.context() as mp:  # the stock runs: every op on its PyTorch path
        mp.setenv("TBAMD_FORCE_REFERENCE", "1")
        m32 = copy.deepcopy(base)
        l32 = _train(m32, data, torch.optim.AdamW(m32.parameters(), lr=1e-3))
        mamp = copy.deepcopy(base)
        lamp = _train(mamp, data, torch.optim.AdamW(mamp.parameters(), lr=1e-3), autocast=True)
    mnat = copy.deepcopy(base).to(torch.bfloat16)
    lnat = _train(mnat, data, FusedAdamW(mnat.parameters(), lr=1e-3), dtype=torch.bfloat16)
    _check(l32, lamp, lnat)
