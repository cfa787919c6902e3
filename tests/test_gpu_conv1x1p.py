"""Persistent 1x1 forward (csrc/conv.hip ``conv1x1_fwd_k``): the expanding 1x1 convs of ResNet
stage 1 (64 -> 256 / 64 -> 128 channels, stride 1) stream pixel tiles through a workgroup that
keeps its weights in registers, and emit one BatchNorm-statistics partial row per stream.
Numerics against a fp32 PyTorch reference of the same conv (torchvision ResNet-50 layers,
ref examples/img_cls/resnet/resnet.py:111 -> cuDNN conv + BN statistics)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402


@pytest.mark.parametrize("N,H,C,K", [(16, 56, 64, 256), (11, 56, 64, 128), (10, 60, 64, 384), (16, 56, 128, 512),
                                     (13, 57, 128, 256)])
def test_conv1x1_persistent_fwd_and_stats(N, H, C, K):
    torch.manual_seed(0)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 1, 1, device="cuda") * 0.1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y, stats = native().conv2d_fwd(x, w, None, 1, 0, False, True)
    ref = F.conv2d(x.float(), w.float())
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err
    # statistics of the STORED bf16 output, summed over the partial rows
    yb = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    s, q = stats[:, 0, :].sum(0), stats[:, 1, :].sum(0)
    assert torch.allclose(s, yb.sum(0), rtol=1e-4, atol=1e-2), (s - yb.sum(0)).abs().max()
    assert torch.allclose(q, yb.square().sum(0), rtol=1e-4, atol=1e-2)
    # and without the statistics epilogue
    y2, none = native().conv2d_fwd(x, w, None, 1, 0, False, False)
    assert torch.equal(y2, y)


def test_conv1x1_persistent_in_bn_model(monkeypatch):
    """A native ResNet-50 forward (stage 1 on the persistent conv, BN statistics from its
    per-stream partial rows) matches the same model with the persistent kernel off (the tiled
    conv, per-tile partial rows) to bf16 summation noise, and is no further from the stock fp32
    ATen forward than that tiled path is."""
    from torchbooster_amd import models

    torch.manual_seed(0)
    m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).train()
    x = torch.randn(16, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    with monkeypatch.context() as mp:
        mp.setenv("TBAMD_FORCE_REFERENCE", "1")
        with torch.no_grad():
            exp = m(x).float()
    outs = {}
    for on in (True, False):
        native().conv_set_persistent_1x1(on)
        m.load_state_dict(state)
        nat = m.to(torch.bfloat16)
        with torch.no_grad():
            outs[on] = nat(x.to(torch.bfloat16)).float()
        m = m.float()
    native().conv_set_persistent_1x1(True)
    rel_on = ((outs[True] - exp).norm() / exp.norm()).item()
    rel_off = ((outs[False] - exp).norm() / exp.norm()).item()
    rel_ab = ((outs[True] - outs[False]).norm() / outs[False].norm()).item()
    print(f"rel vs fp32: persistent {rel_on:.4f} tiled {rel_off:.4f}; persistent vs tiled {rel_ab:.4f}")
    assert rel_on <= 1.25 * rel_off + 0.01, (rel_on, rel_off)
    assert rel_ab < 0.1, rel_ab
