"""BatchNorm finalize folded into the producing conv (csrc/bn_fold.h, conv2d_fwd_bn): the
coefficients, running statistics and batch counter must match the two-launch path (conv
partials -> norm_bn.hip colsum finalize) and the fp32 PyTorch BatchNorm of the same conv output;
repeated launches (arrival counters reset) and run-to-run results are bitwise stable.
Reference: every Conv2d -> BatchNorm2d pair of the ResNet example (examples/img_cls/resnet/
resnet.py:111, torchvision layout)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402

# (N, C, K, H, R, stride): persistent 1x1 (C=64/128), tiled 1x1 / 3x3 with many partial rows
# (two-level fold), few rows (one level), K = 64 tiles, stride 2
SHAPES = [(32, 64, 256, 56, 1, 1), (16, 128, 512, 28, 1, 1), (32, 64, 64, 56, 3, 1), (16, 256, 256, 14, 3, 1),
          (8, 512, 512, 7, 3, 1), (4, 256, 1024, 14, 1, 1), (8, 128, 128, 28, 3, 2), (2, 64, 128, 9, 1, 1)]


def _bf(*s):
    return torch.randn(*s, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("N,C,K,H,R,stride", SHAPES)
def test_conv_fwd_bn_fold_matches_two_launch(N, C, K, H, R, stride):
    torch.manual_seed(0)
    pad = R // 2
    x = _bf(N, C, H, H)
    w = (torch.randn(K, C, R, R, device="cuda") / (R * C ** 0.5)).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    gamma = torch.rand(K, device="cuda") + 0.5
    beta = torch.randn(K, device="cuda")
    rm0, rv0 = torch.randn(K, device="cuda"), torch.rand(K, device="cuda") + 0.5
    mom, eps = 0.1, 1e-5
    # two-launch path
    y_ref, stats = native().conv2d_fwd(x, w, None, stride, pad, False, True)
    rm1, rv1, nbt1 = rm0.clone(), rv0.clone(), torch.zeros((), dtype=torch.long, device="cuda")
    rows = y_ref.permute(0, 2, 3, 1).reshape(-1, K)
    mean1, invstd1, scale1, shift1 = native().bn_stats(rows, stats, gamma, beta, rm1, rv1, True, mom, eps, nbt1)
    # folded
    rm2, rv2, nbt2 = rm0.clone(), rv0.clone(), torch.zeros((), dtype=torch.long, device="cuda")
    y, coeff = native().conv2d_fwd_bn(x, w, stride, pad, gamma, beta, rm2, rv2, nbt2, mom, eps)
    assert torch.equal(y, y_ref)
    for a, b in ((coeff[0], mean1), (coeff[1], invstd1), (coeff[2], scale1), (coeff[3], shift1), (rm2, rm1),
                 (rv2, rv1)):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()
    assert int(nbt2) == 1 == int(nbt1)
    # fp32 BatchNorm of the same stored output
    yf = y.float()
    m = yf.mean(dim=(0, 2, 3))
    v = yf.var(dim=(0, 2, 3), unbiased=False)
    assert torch.allclose(coeff[0], m, rtol=1e-4, atol=1e-4)
    assert torch.allclose(coeff[1], (v + eps).rsqrt(), rtol=1e-3, atol=1e-4)
    # repeated launches: counters back at zero, bitwise identical coefficients
    for _ in range(3):
        y3, c3 = native().conv2d_fwd_bn(x, w, stride, pad, gamma, beta, None, None, None, mom, eps)
        assert torch.equal(y3, y) and torch.equal(c3, coeff)


def test_resnet50_step_fold_on_off(monkeypatch):
    """One training forward/backward of ResNet-50 (b16, 112 px) with the fold on vs off: same loss,
    same running statistics (to float rounding of the summation order), same gradients."""
    from torchbooster_amd import models
    from torchbooster_amd.ops import conv as CV

    def run(fold):
        monkeypatch.setattr(CV, "_FOLD_BN", fold)
        torch.manual_seed(0)
        m = models.resnet50(num_classes=10).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last).train()
        x = torch.randn(16, 3, 112, 112, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        t = torch.randint(0, 10, (16,), device="cuda")
        loss = F.cross_entropy(m(x).float(), t)
        loss.backward()
        torch.cuda.synchronize()
        bufs = [b.detach().float().clone() for n, b in m.named_buffers() if "running" in n]
        nbt = [int(b) for n, b in m.named_buffers() if "num_batches" in n]
        grads = torch.cat([p.grad.float().reshape(-1) for p in m.parameters()])
        return loss.item(), bufs, nbt, grads

    torch.backends.cudnn.deterministic = True
    l0, b0, n0, g0 = run(False)
    l1, b1, n1, g1 = run(True)
    assert abs(l0 - l1) <= 1e-3 * max(1.0, abs(l0)), (l0, l1)
    assert n0 == n1 and all(v == 1 for v in n1)
    for a, b in zip(b0, b1):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5)
    rel = ((g0 - g1).norm() / g0.norm()).item()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("N,C,K,H,R,stride", [(16, 64, 64, 56, 3, 1), (8, 256, 64, 56, 1, 1), (16, 128, 128, 28, 3, 2),
                                              (8, 256, 512, 14, 1, 2), (2, 64, 128, 9, 3, 1)])
def test_dgrad_bnb_fold_matches_two_launch(N, C, K, H, R, stride):
    """Backward: the dgrad's BN-backward partials finalized in its tail (dgamma, dbeta, apply
    coefficients) == the separate finalize (norm_bn.hip bn_backward_from_partials)."""
    torch.manual_seed(1)
    pad = R // 2
    P = (H + 2 * pad - R) // stride + 1
    dy = _bf(N, K, P, P)
    w = (torch.randn(K, C, R, R, device="cuda") / (R * C ** 0.5)).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    wt = native().conv_flip_weight(w)
    xb = _bf(N, C, H, H)  # the BN input of the conv's input x = relu(bn(xb))
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.randn(C, device="cuda") * 0.1
    mean = torch.randn(C, device="cuda") * 0.1
    invstd = torch.rand(C, device="cuda") + 0.5
    scale = gamma * invstd
    shift = beta - mean * scale
    if stride == 1:
        args = (dy, wt, None, 1, R - 1 - pad, False, False, None, None, 1, xb, scale, shift, mean, None)
        call = native().conv2d_fwd
    else:
        args = (dy, wt, R, R, pad, H, H, 1, xb, scale, shift, mean, None)
        call = native().conv2d_dgrad_s2
    dx, part = call(*args)[:2]
    outs = call(*args, fold_invstd=invstd, fold_gamma=gamma, fold_training=True)
    assert len(outs) == 5
    assert torch.equal(outs[0], dx)
    coef, dg, db = outs[2], outs[3], outs[4]
    rows = xb.permute(0, 2, 3, 1).reshape(-1, C)
    dz_rows = dx.permute(0, 2, 3, 1).reshape(-1, C)
    ref_dx, ref_dg, ref_db, _ = native().bn_backward_from_partials(dz_rows, rows, part, gamma, mean, invstd, scale,
                                                                  shift, True, 1, 0.01, None, None, None, False)
    assert torch.allclose(dg, ref_dg, rtol=1e-5, atol=1e-5), (dg - ref_dg).abs().max()
    assert torch.allclose(db, ref_db, rtol=1e-5, atol=1e-5), (db - ref_db).abs().max()
    got_dx, _ = native().bn_backward_apply_coef(dz_rows, rows, coef, scale, shift, 1, 0.01)
    diff = (got_dx.float() - ref_dx.float()).abs().max().item()
    assert diff <= 1e-2 * ref_dx.float().abs().max().item() + 1e-6, diff
    # slots as outputs, repeated launches
    gs, bs = torch.empty_like(dg), torch.empty_like(db)
    for _ in range(2):
        o2 = call(*args, fold_invstd=invstd, fold_gamma=gamma, fold_training=True, fold_dgamma=gs, fold_dbeta=bs)
        assert o2[3].data_ptr() == gs.data_ptr() and torch.equal(gs, dg) and torch.equal(bs, db)
        assert torch.equal(o2[2], coef)
