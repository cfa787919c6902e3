"""ResidualGradLink carrier (ops/norm.py): in a bottleneck with a downsample branch, the block-output
BatchNorm hands (dy, ReLU mask) to the downsample BN, whose backward applies the mask itself
(csrc/norm_bn.hip MASKIN with no activation) instead of reading a written dy * mask.  Gradients
must match the model without the link; a modified branch gradient must fail loudly."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.models import resnet as R  # noqa: E402
from torchbooster_amd.ops import _ext  # noqa: E402


def _grads(model, x, on, monkeypatch):
    monkeypatch.setattr(R, "_RES_CARRIER", on)
    model.zero_grad(set_to_none=True)
    model(x).float().square().mean().backward()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None}


def test_carrier_matches_written_residual_gradient(monkeypatch):
    _ext.native()
    torch.manual_seed(0)
    model = R.resnet50(num_classes=16).cuda().to(torch.bfloat16)
    x = torch.randn(4, 3, 64, 64, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    on = _grads(model, x, True, monkeypatch)
    off = _grads(model, x, False, monkeypatch)
    assert on.keys() == off.keys()
    worst = 0.0
    for n in on:
        d = ((on[n] - off[n]).norm() / off[n].norm().clamp_min(1e-12)).item()
        worst = max(worst, d)
        assert d < 1e-3, (n, d)
    # the downsample branches really took the carrier path: their BN gradients exist and are nonzero
    assert any("down.bn" in n and on[n].abs().sum() > 0 for n in on), worst


def test_carrier_fails_loudly_on_modified_gradient(monkeypatch):
    _ext.native()
    monkeypatch.setattr(R, "_RES_CARRIER", True)
    torch.manual_seed(1)
    model = R.resnet50(num_classes=16).cuda().to(torch.bfloat16)
    x = torch.randn(2, 3, 64, 64, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    blk = model.layer1[0]
    assert blk.down is not None
    def hook(mod, inp, out):
        out.register_hook(lambda g: g * 1.0)  # a different tensor reaches the downsample BN
        # (returns None: the module output itself is unchanged)

    h = blk.down.register_forward_hook(hook)
    try:
        with pytest.raises(RuntimeError, match="carrier"):
            model(x).float().square().mean().backward()
    finally:
        h.remove()
