"""Model zoo: parameter counts match the reference architectures and
CPU forward/backward works through the reference (ATen) paths of the fused ops."""
import pytest
import torch
import torch.nn.functional as F

from torchbooster_amd import models as M


def n(m):
    return sum(p.numel() for p in m.parameters())


def test_param_counts_match_reference():
    assert n(M.lenet()) == 44_470
    assert n(M.MLPGenerator()) == 730_896
    assert n(M.MLPDiscriminator()) == 665_089
    assert n(M.VAE()) == 1_526_800
    assert n(M.vgg19().features) == 20_024_384
    assert n(M.StyleNet()) == 496_515  # weight-tied residual x5 (A.2 B19)
    assert n(M.AdaINDecoder()) == 2_931_267
    assert n(M.resnet50()) == 25_557_032
    r18 = M.resnet18(num_classes=10)
    assert n(r18) == 11_181_642
    assert n(M.vit_b_16()) == 86_567_656


def test_vgg_indexing_matches_torchvision_layout():
    f = M.vgg19().features
    assert isinstance(f[0], torch.nn.Conv2d) and isinstance(f[4], torch.nn.MaxPool2d)
    assert isinstance(f[28], torch.nn.Conv2d) and isinstance(f[29], torch.nn.ReLU)
    assert len(f) == 37


@pytest.mark.parametrize("name,shape", [("resnet18", (2, 3, 32, 32)), ("lenet", (2, 1, 28, 28)),
                                        ("vit_tiny", (2, 3, 32, 32))])
def test_forward_backward_cpu(name, shape):
    m = getattr(M, name)(num_classes=10)
    x = torch.randn(*shape)
    y = m(x)
    assert y.shape == (2, 10)
    F.cross_entropy(y, torch.tensor([1, 2])).backward()
    assert all(p.grad is not None for p in m.parameters() if p.requires_grad)


def test_style_models_and_losses():
    from torchbooster_amd.models.style import adain, gram_matrix, gram_matrix_flat, total_variation

    x = torch.randn(2, 3, 32, 32)
    assert M.StyleNet()(x).shape == x.shape
    f = torch.randn(2, 8, 5, 5)
    g = gram_matrix(f)
    ref = torch.bmm(f.view(2, 8, 25), f.view(2, 8, 25).transpose(1, 2)) / (8 * 25)
    assert torch.allclose(g, ref, atol=1e-6)
    g2 = gram_matrix(f.contiguous(memory_format=torch.channels_last))
    assert torch.allclose(g2, ref, atol=1e-5)
    f1 = torch.randn(1, 8, 5, 5)
    assert torch.allclose(gram_matrix_flat(f1.contiguous(memory_format=torch.channels_last)),
                          gram_matrix_flat(f1), atol=1e-5)
    assert total_variation(torch.zeros(1, 3, 4, 4)).item() == 0
    out = adain(torch.randn(2, 4, 6, 6), torch.randn(2, 4, 6, 6))
    assert out.shape == (2, 4, 6, 6)


def test_dcgan_shapes():
    g, d = M.dcgan128(z_dim=16, width=8)
    img = g(torch.randn(3, 16))
    assert img.shape == (3, 3, 128, 128)
    assert d(img).shape == (3, 1)


def test_groupnorm_layernorm_reference_paths():
    from torchbooster_amd.ops.norm import GroupNormAct, InstanceNormAct2d, LayerNorm

    x = torch.randn(2, 8, 4, 4)
    assert torch.allclose(InstanceNormAct2d(8)(x), torch.nn.InstanceNorm2d(8, affine=True)(x), atol=1e-5)
    assert torch.allclose(GroupNormAct(2, 8)(x), torch.nn.GroupNorm(2, 8)(x), atol=1e-5)
    ln = LayerNorm(16)
    t = torch.randn(3, 5, 16)
    r = torch.randn(3, 5, 16)
    y, s = ln(t, r)
    assert torch.allclose(s, t + r) and torch.allclose(y, F.layer_norm(t + r, (16,)), atol=1e-5)


def test_torchvision_layout_weights_roundtrip(tmp_path):
    """A torchvision-layout state dict (saved by torchvision's own key scheme) loads into
    models.tv with strict=True; the reference's fine-tune (1000-class weights into a
    10-class head, resnet.py:111-112) loads with the head skipped."""
    import torch

    from torchbooster_amd.models import load_weights, tv, vgg19

    src = tv.resnet18(num_classes=1000)
    keys = list(src.state_dict())
    assert keys[:6] == ["conv1.weight", "bn1.weight", "bn1.bias", "bn1.running_mean", "bn1.running_var",
                        "bn1.num_batches_tracked"]
    assert "layer2.0.downsample.0.weight" in keys and "layer4.1.bn2.weight" in keys and keys[-1] == "fc.bias"
    p = tmp_path / "resnet18.pth"
    torch.save({"state_dict": {"module." + k: v for k, v in src.state_dict().items()}}, p)
    full = load_weights(tv.resnet18(num_classes=1000), p)
    for k, v in src.state_dict().items():
        assert torch.equal(full.state_dict()[k], v), k
    head = tv.resnet18(num_classes=10, weights=str(p))
    assert torch.equal(head.layer3[1].conv2.weight, src.layer3[1].conv2.weight)
    assert head.fc.weight.shape == (10, 512)
    v = vgg19()
    q = tmp_path / "vgg19.pth"
    torch.save(v.state_dict(), q)
    w = load_weights(vgg19(), q)
    assert torch.equal(w.features[28].weight, v.features[28].weight)
