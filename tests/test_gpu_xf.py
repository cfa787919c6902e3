"""BatchNorm + ReLU applied inside the consumer conv's operand staging (csrc/xf.h): the forward
(persistent 1x1 kernel) and the weight gradient (1x1 and 3x3, stride 1 / 2 with padded taps,
partial pixel tiles) over relu(x * scale + shift) must equal -- bitwise -- the same kernels run on the
materialised BN output (norm_bn.hip apply, the same fmaf arithmetic), and follow fp32 PyTorch.
Reference: the bottleneck's bn1 -> conv2 and bn2 -> conv3 (examples/img_cls/resnet/resnet.py:111,
torchvision Bottleneck)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402

# the forward: the persistent 1x1 shapes (C = 64 / 128, K % 128, >= 32768 pixels)
FWD_SHAPES = [(16, 64, 256, 56, 1, 1), (48, 128, 512, 28, 1, 1), (11, 64, 128, 57, 1, 1)]
# (N, C, K, H, R, stride) of the weight gradient: 1x1, 3x3 s1 / s2, ragged pixel tiles
SHAPES = [(16, 64, 256, 56, 1, 1), (8, 128, 512, 28, 1, 1), (8, 256, 1024, 14, 1, 1), (8, 64, 64, 56, 3, 1),
          (8, 128, 128, 28, 3, 2), (4, 256, 256, 14, 3, 1), (3, 64, 128, 13, 3, 1), (2, 512, 512, 7, 3, 1)]


def _bf(*s):
    return torch.randn(*s, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _coeffs(C):
    sc = (torch.rand(C, device="cuda") + 0.5).contiguous()
    sh = (torch.randn(C, device="cuda") * 0.5).contiguous()
    coeff = torch.stack([torch.zeros_like(sc), torch.ones_like(sc), sc, sh]).contiguous()
    return sc, sh, coeff


def _apply(x, coeff):
    N, C, H, W = x.shape
    rows = x.permute(0, 2, 3, 1).reshape(-1, C)
    a, _ = native().bn_apply_coeff(rows, coeff, None, 1, 0.01, False)
    return a.view(N, H, W, C).permute(0, 3, 1, 2)


@pytest.mark.parametrize("N,C,K,H,R,stride", FWD_SHAPES)
def test_conv_fwd_xf_matches_materialised_bn(N, C, K, H, R, stride):
    torch.manual_seed(0)
    pad = R // 2
    x = _bf(N, C, H, H)
    w = (torch.randn(K, C, R, R, device="cuda") / (R * C ** 0.5)).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    sc, sh, coeff = _coeffs(C)
    a = _apply(x, coeff)
    y_ref, st_ref = native().conv2d_fwd(a, w, None, stride, pad, False, True)
    y, st = native().conv2d_fwd_xf(x, w, sc, sh, stride, pad, True)
    assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max()
    assert torch.equal(st, st_ref)
    ref = F.conv2d(F.relu(x.float() * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)), w.float(), None, stride, pad)
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("N,C,K,H,R,stride", SHAPES)
def test_conv_wgrad_xf_matches_materialised_bn(N, C, K, H, R, stride):
    torch.manual_seed(1)
    pad = R // 2
    P = (H + 2 * pad - R) // stride + 1
    x = _bf(N, C, H, H)
    dy = _bf(N, K, P, P)
    sc, sh, coeff = _coeffs(C)
    a = _apply(x, coeff)
    dw_ref = native().conv2d_wgrad(dy, a, R, R, stride, pad)
    dw = native().conv2d_wgrad_xf(dy, x, sc, sh, R, R, stride, pad)
    assert torch.equal(dw, dw_ref), (dw.float() - dw_ref.float()).abs().max()


def test_resnet50_lazy_bn_matches_materialised(monkeypatch):
    """The bottleneck's bn1 -> conv2 and bn2 -> conv3 with the BN + ReLU outputs never written
    (models/resnet.py _lazy_ok, ops.norm.LazyAct: bn2 -> conv3 where conv3 is a persistent 1x1) == the
    materialised path:
    loss and running statistics bitwise equal, and gradients no further from the stock fp32 ATen
    step than the materialised path's.  The forward route is pinned to the native kernels: the
    materialised conv3 then runs the same persistent 1x1 kernel (same fmaf arithmetic) as the XF
    one.  Left to the per-box timing, a big-tile / MIOpen route could win conv3's shape, and the
    53-BN chain turns its different bf16 rounding into running-statistics deviations of either
    sign (one box in round 6: 1.6e-3 on a near-zero mean, vs 0 with the pinned route,
    scripts/tools/xf_buffer_probe.py)."""
    import torch.nn.functional as F

    from torchbooster_amd import models
    from torchbooster_amd.models import resnet as RN

    calls = [0]
    orig = RN.conv2d_xf_bn_stats

    def counted(*a, **k):
        calls[0] += 1
        return orig(*a, **k)

    monkeypatch.setattr(RN, "conv2d_xf_bn_stats", counted)
    torch.manual_seed(0)
    m0 = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).train()
    state = {k: v.clone() for k, v in m0.state_dict().items()}
    x = torch.randn(48, 3, 160, 160, device="cuda").contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (48,), device="cuda")

    # (this test isolates BN-in-operand: the lazy affine downsample output, checked against fp32 in
    # tests/test_gpu_res_carrier.py, stays off so both runs share every other rounding)
    monkeypatch.setattr(RN, "_LAZY_DS", False)
    from torchbooster_amd.ops import conv as CV

    monkeypatch.setitem(CV._FORCE, "fwd", "native")

    def run(lazy, dtype=torch.bfloat16):
        monkeypatch.setattr(RN, "_LAZY_BN", lazy)
        m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).train()
        m.load_state_dict(state)
        m = m.to(dtype)
        loss = F.cross_entropy(m(x.to(dtype)).float(), t)
        loss.backward()
        torch.cuda.synchronize()
        bufs = [b.detach().float().clone() for n, b in m.named_buffers() if "running" in n]
        grads = torch.cat([p.grad.float().reshape(-1) for p in m.parameters()])
        return loss.item(), bufs, grads

    with monkeypatch.context() as mp:
        mp.setenv("TBAMD_FORCE_REFERENCE", "1")
        _, _, gref = run(False, torch.float32)
    calls[0] = 0
    l0, b0, g0 = run(False)
    assert calls[0] == 0
    l1, b1, g1 = run(True)
    assert calls[0] == 3, calls[0]  # stage 1: 48 x 40 x 40 conv3 pixels (stage 2's 19,200 are too few)
    assert l0 == l1, (l0, l1)
    for a, b in zip(b0, b1):
        assert torch.equal(a, b), ((a - b).abs().max().item(), a.abs().max().item())
    assert torch.isfinite(g1).all()
    rel0 = ((g0 - gref).norm() / gref.norm()).item()
    rel1 = ((g1 - gref).norm() / gref.norm()).item()
    print(f"grad rel vs fp32: materialised {rel0:.4f} lazy {rel1:.4f}")
    assert rel1 <= 1.25 * rel0 + 0.01, (rel1, rel0)


def test_resnet50_lazy_bn2_persistent_only_default(monkeypatch):
    """The default: only bn2 -> conv3 of the bottlenecks whose conv3 runs on the
    persistent 1x1 kernel (stage 1 and 2 at this size) are lazy; one training step stays finite
    and its loss matches the materialised path."""
    import torch.nn.functional as F

    from torchbooster_amd import models
    from torchbooster_amd.models import resnet as RN

    calls = [0]
    orig = RN.conv2d_xf_bn_stats

    def counted(*a, **k):
        calls[0] += 1
        return orig(*a, **k)

    monkeypatch.setattr(RN, "conv2d_xf_bn_stats", counted)
    torch.manual_seed(0)
    m = models.resnet50(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last).train()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(48, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (48,), device="cuda")
    losses = {}
    for on in (False, True):
        monkeypatch.setattr(RN, "_LAZY_BN", on)
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x).float(), t)
        loss.backward()
        torch.cuda.synchronize()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters())
        losses[on] = loss.item()
    assert calls[0] == 3 + 4, calls[0]  # stage 1 (C = 64) and stage 2 (C = 128) bottlenecks
    assert abs(losses[True] - losses[False]) <= 1e-2 * max(1.0, abs(losses[False])), losses


def test_lazy_bn_off_under_forward_hooks(monkeypatch):
    """A forward hook on a bottleneck's bn2 must see the real activation: the lazy path is skipped
    for that block (models/resnet.py _lazy_ok)."""
    import torch.nn.functional as F

    from torchbooster_amd import models
    from torchbooster_amd.models import resnet as RN

    monkeypatch.setattr(RN, "_LAZY_BN", True)
    torch.manual_seed(0)
    m = models.resnet50(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last).train()
    seen = []
    blk = m.layer1[0]
    blk.c2.bn.register_forward_hook(lambda mod, i, o: seen.append(o.detach().float().clone()))
    # 48 x 28 x 28 conv3 pixels: layer1's bn2 -> conv3 would be lazy without the hook
    x = torch.randn(48, 3, 112, 112, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    F.cross_entropy(m(x).float(), torch.randint(0, 10, (48,), device="cuda")).backward()
    assert len(seen) == 1 and seen[0].std() > 0  # a placeholder would be one repeated value
    assert torch.isfinite(seen[0]).all() and (seen[0] >= 0).all() and seen[0].abs().sum() > 0


def test_conv_fwd_xf_refuses_tiled_shapes():
    """The BN-in-operand forward exists for the persistent 1x1 kernel only: other shapes are
    refused loudly (the caller materialises the activation instead)."""
    x = _bf(8, 256, 14, 14)
    w = _bf(256, 256, 3, 3)
    sc, sh, _ = _coeffs(256)
    assert not native().conv_fwd_xf_supported(8 * 14 * 14, 256, 256, 3, 3, 1, 1)
    with pytest.raises(RuntimeError, match="persistent 1x1"):
        native().conv2d_fwd_xf(x, w, sc, sh, 1, 1, True)
