"""CPU paths of ops/losses.py and ops/resample.py: the PyTorch references the GPU kernels are tested against."""
import torch
import torch.nn.functional as F

from torchbooster_amd.models.style import mu_std, total_variation
from torchbooster_amd.ops import losses as L
from torchbooster_amd.ops.resample import ReflectionPad2d, UpsampleNearest2d, reflection_pad2d, upsample_nearest2d


def test_total_variation_matches_reference_formula():
    torch.manual_seed(0)
    x = torch.randn(2, 3, 9, 7)
    ref = (x[:, :, :, :-1] - x[:, :, :, 1:]).abs().sum() + (x[:, :, :-1, :] - x[:, :, 1:, :]).abs().sum()
    assert torch.allclose(total_variation(x), ref)
    assert torch.allclose(L.total_variation(x.contiguous(memory_format=torch.channels_last)), ref)


def test_hinge_bce_kld_reference_values():
    x = torch.tensor([[-2.0], [0.5], [3.0]])
    assert torch.allclose(L.hinge(x, 1.0, -1.0), torch.tensor((3.0 + 0.5 + 0.0) / 3))
    assert torch.allclose(L.hinge(x, 1.0, 1.0), torch.tensor((0.0 + 1.5 + 4.0) / 3))
    t = torch.rand(4, 5)
    z = torch.randn(4, 5)
    assert torch.allclose(L.bce_with_logits(z, t), F.binary_cross_entropy_with_logits(z, t))
    mu, lv = torch.zeros(4, 3), torch.zeros(4, 3)
    assert L.gaussian_kld(mu, lv).item() == 0.0
    mu = torch.ones(4, 3)
    assert torch.allclose(L.gaussian_kld(mu, lv), torch.tensor(1.5))


def test_mean_std_expanded_like_adain():
    torch.manual_seed(1)
    f = torch.randn(2, 4, 5, 6)
    mu, std = mu_std(f)
    assert mu.shape == f.shape and std.shape == f.shape
    assert torch.allclose(mu[:, :, 0, 0], f.mean(dim=[2, 3]))
    assert torch.allclose(std[:, :, 3, 2], (f.var(dim=[2, 3]) + 1e-5).sqrt())


def test_resample_modules_match_torch():
    torch.manual_seed(2)
    x = torch.randn(2, 3, 6, 5)
    assert torch.equal(ReflectionPad2d(2)(x), torch.nn.ReflectionPad2d(2)(x))
    assert torch.equal(reflection_pad2d(x, (1, 2, 0, 3)), F.pad(x, (1, 2, 0, 3), mode="reflect"))
    assert torch.equal(UpsampleNearest2d(2)(x), torch.nn.Upsample(scale_factor=2)(x))
    assert torch.equal(upsample_nearest2d(x, 3), F.interpolate(x, scale_factor=3, mode="nearest"))


def _rpad_gather_backward(dy, H, W, pads):
    """Python model of csrc/aux_ops.hip rpad_bwd_k's source-index gather."""
    pl, pr, pt, pb = pads

    def src(i, n, p, pe):
        o = [i + p]
        if 1 <= i <= p:
            o.append(p - i)
        if n - 1 - pe <= i <= n - 2:
            o.append(p + 2 * (n - 1) - i)
        return o

    dx = torch.zeros(dy.size(0), dy.size(1), H, W)
    for h in range(H):
        for w in range(W):
            for oh in src(h, H, pt, pb):
                for ow in src(w, W, pl, pr):
                    dx[:, :, h, w] += dy[:, :, oh, ow]
    return dx


def test_reflection_pad_gather_backward_model():
    torch.manual_seed(3)
    for (H, W), pads in [((6, 7), (2, 3, 1, 4)), ((3, 3), (2, 2, 2, 2)), ((5, 4), (0, 1, 3, 0))]:
        x = torch.randn(1, 2, H, W, requires_grad=True)
        y = F.pad(x, pads, mode="reflect")
        g = torch.randn_like(y)
        y.backward(g)
        assert torch.allclose(_rpad_gather_backward(g, H, W, pads), x.grad, atol=1e-6)


def test_conv_transpose_module_cpu_fallback():
    from torchbooster_amd.ops.conv import ConvTranspose2d

    torch.manual_seed(4)
    m = ConvTranspose2d(8, 4, 4, 2, 1)
    ref = torch.nn.ConvTranspose2d(8, 4, 4, 2, 1)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 8, 5, 5)
    assert torch.allclose(m(x), ref(x))


def test_style_stats_loss_equals_expanded_mse():
    """style_stats_loss == the reference's mse over expanded mean/std (adain.py:55-58, 134)."""
    from torchbooster_amd.models.style import style_stats_loss

    torch.manual_seed(0)
    m = [torch.randn(2, 8, 5, 6, requires_grad=True), torch.randn(2, 4, 3, 3, requires_grad=True)]
    s = [torch.randn(2, 8, 5, 6), torch.randn(2, 4, 3, 3)]
    ref = sum(F.mse_loss(xm, sm) + F.mse_loss(xs, ss) for (xm, xs), (sm, ss) in zip(map(mu_std, m), map(mu_std, s)))
    new = style_stats_loss(m, s)
    assert torch.allclose(ref, new, rtol=1e-6, atol=0)
    for a, b in zip(torch.autograd.grad(ref, m), torch.autograd.grad(new, m)):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-8)
