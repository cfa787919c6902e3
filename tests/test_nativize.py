"""nativize(): stock torch.nn models rewritten onto the native modules (CPU:
structure, state-dict keys, identical outputs/grads through the ATen paths)."""
import copy

import torch
import torch.nn as nn

from torchbooster_amd.config import EnvironementConfig
from torchbooster_amd.nativize import nativize
from torchbooster_amd.ops.conv import Conv2d
from torchbooster_amd.ops.linear import Linear, LinearGELU
from torchbooster_amd.ops.norm import BatchNormAct2d, InstanceNormAct2d
from torchbooster_amd.utils import nativize as utils_nativize


def lenet():
    """/root/reference/examples/img_cls/lenet/lenet.py:29-36, literally."""
    return nn.Sequential(
        nn.Conv2d(1, 6, 5, 1), nn.BatchNorm2d(6), nn.GELU(), nn.MaxPool2d(2, 2),
        nn.Conv2d(6, 16, 5, 1), nn.BatchNorm2d(16), nn.GELU(), nn.MaxPool2d(2, 2),
        nn.Flatten(), nn.Linear(256, 120), nn.GELU(), nn.Linear(120, 84), nn.GELU(), nn.Linear(84, 10))


class BasicBlock(nn.Module):
    """torchvision.models.resnet.BasicBlock, stock modules (torchvision is not installed)."""

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


def resnet18(num_classes=10):
    layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
              nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        layers += [BasicBlock(cin, cout, stride), BasicBlock(cout, cout)]
        cin = cout
    return nn.Sequential(*layers, nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, num_classes))


def _check_same(model, make_x, steps=2):
    torch.manual_seed(0)
    ref = copy.deepcopy(model)
    keys = sorted(model.state_dict().keys())
    nat = nativize(model)
    assert sorted(nat.state_dict().keys()) == keys
    for _ in range(steps):
        x = make_x()
        a, b = nat(x), ref(x)
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-5)
        a.square().mean().backward()
        b.square().mean().backward()
    for (n1, p1), (n2, p2) in zip(nat.named_parameters(), ref.named_parameters()):
        assert n1 == n2 and torch.allclose(p1.grad, p2.grad, atol=1e-5, rtol=1e-4), n1
    return nat


def _calls(mod):
    """call_module nodes of a container's fused forward graph."""
    return [n for n in mod._tb_fused_graph.graph.nodes if n.op == "call_module"]


def test_lenet_sequential_is_nativized_and_fused():
    nat = _check_same(lenet(), lambda: torch.randn(8, 1, 28, 28))
    mods = dict(nat.named_modules())
    assert type(nat) is nn.Sequential  # same object / class: no GraphModule
    assert isinstance(mods["0"], Conv2d) and isinstance(mods["1"], BatchNormAct2d)
    assert mods["1"].act == "none" and type(mods["9"]) is Linear  # leaves keep their own behaviour
    calls = {n.target: n.kwargs for n in _calls(nat)}
    assert calls["1"] == {"act": "gelu", "slope": 0.01} and calls["9"] == {"act": "gelu"}
    assert "2" not in calls and "10" not in calls  # GELUs absorbed into the fused forward
    x = torch.randn(4, 6, 24, 24)
    assert torch.equal(nat[1](x), nn.functional.batch_norm(x, None, None, nat[1].weight, nat[1].bias, True))


def test_resnet18_blocks_fuse_residual_tails():
    nat = _check_same(resnet18(), lambda: torch.randn(2, 3, 64, 64))
    blocks = [m for m in nat.modules() if isinstance(m, BasicBlock)]
    assert len(blocks) == 8 and all(getattr(b, "_tb_nativized", False) for b in blocks)
    assert all(b.bn2.act == "none" and b.relu.inplace for b in blocks)  # unchanged leaves
    stem = {n.target: n.kwargs for n in _calls(nat)}
    assert stem["1"]["act"] == "relu" and "2" not in stem  # stem BN + ReLU fused in the outer Sequential


def test_instance_norm_and_untraceable_models():
    class Dyn(nn.Module):  # data-dependent control flow: leaf swaps only
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 8, 3, padding=1)
            self.norm = nn.InstanceNorm2d(8, affine=True)
            self.act = nn.GELU()

        def forward(self, x):
            y = self.act(self.norm(self.conv(x)))
            return y if float(y.sum()) > -1e9 else -y

    m = Dyn()
    nat = _check_same(m, lambda: torch.randn(2, 3, 16, 16))
    assert isinstance(nat.norm, InstanceNormAct2d) and isinstance(nat.conv, Conv2d)


def test_env_make_applies_nativize_only_on_gpu():
    env = EnvironementConfig(n_gpu=0)
    m = env.make(lenet())
    assert type(m[0]) is nn.Conv2d  # CPU: untouched
    assert utils_nativize is nativize
    assert EnvironementConfig().native is True


def test_pad_and_upsample_fold_into_conv():
    """StyleNet / AdaIN ``Conv`` (ReflectionPad2d -> Conv2d) and ``DeconvIN`` (Upsample ->
    ReflectionPad2d -> Conv2d) chains become single convs with the padding / upsampling in
    their addressing (``fold=`` per call); same state-dict keys, same outputs and gradients."""
    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.block = nn.Sequential(nn.ReflectionPad2d(4), nn.Conv2d(3, 8, 9), nn.InstanceNorm2d(8, affine=True),
                                       nn.GELU(), nn.Upsample(scale_factor=2, mode="nearest"), nn.ReflectionPad2d(1),
                                       nn.Conv2d(8, 3, 3), nn.Upsample(scale_factor=2), nn.Conv2d(3, 4, 3, padding=1))

        def forward(self, x):
            return self.block(x)

    nat = _check_same(Net(), lambda: torch.randn(2, 3, 16, 16))
    calls = {n.target: n.kwargs for n in _calls(nat.block)}
    assert list(calls) == ["1", "2", "6", "8"]
    assert calls["1"] == {"fold": (4, True, 1)} and calls["6"] == {"fold": (1, True, 2)}
    assert calls["8"] == {"fold": (1, False, 2)} and calls["2"]["act"] == "gelu"
    assert not hasattr(nat.block[1], "_tb_fold")  # the conv itself is untouched


def test_same_and_asymmetric_padding_are_not_folded():
    """``padding='same'`` / asymmetric pads after Upsample or ReflectionPad used to
    be folded as padding 0 (wrong values / shape)."""
    net = nn.Sequential(nn.Upsample(scale_factor=2), nn.Conv2d(3, 4, 3, padding="same"),
                        nn.ReflectionPad2d((0, 1, 0, 1)), nn.Conv2d(4, 4, 3, padding=(0, 1)),
                        nn.Upsample(scale_factor=2), nn.Conv2d(4, 2, 3, padding=(1, 0)))
    nat = _check_same(net, lambda: torch.randn(2, 3, 8, 8))
    assert not getattr(nat, "_tb_nativized", False)  # nothing to fold: forward untouched


class _VAE(nn.Module):
    """The reference VAE's shape (vae.py:30-60): custom attributes and methods used after env.make."""

    def __init__(self):
        super().__init__()
        self.z_dim = 4
        self.encoder = nn.Sequential(nn.Linear(16, 32), nn.GELU(), nn.Linear(32, 8))
        self.decoder = nn.Sequential(nn.Linear(4, 32), nn.GELU(), nn.Linear(32, 16), nn.Sigmoid())

    def forward(self, x):
        mu, logvar = self.encoder(x).chunk(2, dim=-1)
        return self.decoder(mu), mu, logvar


def test_custom_methods_survive_and_leaves_stay_stock():
    torch.manual_seed(0)
    vae = _VAE()
    ref = copy.deepcopy(vae)
    nat = nativize(vae)
    assert nat is vae and nat.z_dim == 4 and type(nat.decoder) is nn.Sequential
    z = torch.randn(5, 4)
    assert torch.allclose(nat.decoder(z), ref.decoder(z), atol=1e-6)  # no double GELU
    lin = nat.decoder[0]
    assert torch.allclose(lin(z), ref.decoder[0](z), atol=1e-6)  # the leaf alone: no GELU
    assert getattr(nat.decoder, "_tb_nativized", False)
    x = torch.randn(3, 16)
    for a, b in zip(nat(x), ref(x)):
        assert torch.allclose(a, b, atol=1e-6)
    c = copy.deepcopy(nat)  # deep copies keep working (and stay independent)
    assert torch.allclose(c.decoder(z), ref.decoder(z), atol=1e-6)
    with torch.no_grad():
        c.decoder[0].weight.zero_()
    assert not torch.allclose(c.decoder(z), nat.decoder(z))


def test_training_branches_and_attribute_stores_are_not_traced():
    class Branchy(nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(4, 4)
            self.act = nn.GELU()

        def forward(self, x):
            y = self.act(self.lin(x))
            return y * 2 if self.training else y

    class Stores(nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(4, 4)
            self.act = nn.GELU()

        def forward(self, x):
            self.last = self.lin(x)
            return self.act(self.last)

    b, s = nativize(Branchy()), nativize(Stores())
    assert not getattr(b, "_tb_nativized", False) and not getattr(s, "_tb_nativized", False)
    b.eval()
    x = torch.randn(2, 4)
    assert torch.allclose(b(x), nn.functional.gelu(b.lin(x)))
    s(x)
    assert hasattr(s, "last")


def test_hooks_registered_after_nativize_fire():
    nat = nativize(lenet())
    seen = []
    nat[2].register_forward_hook(lambda m, i, o: seen.append(o.shape))
    nat(torch.randn(2, 1, 28, 28))
    assert seen == [torch.Size([2, 6, 24, 24])]


class _TVBottleneck(nn.Module):
    """torchvision.models.resnet.Bottleneck, stock modules."""

    def __init__(self, cin, width, stride=1):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class TVResNet(nn.Module):
    """torchvision.models.resnet.ResNet layout (conv1 .. fc), stock modules."""

    def __init__(self, layers=(1, 1, 1, 1), num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        for i, n in enumerate(layers):
            blocks = []
            for j in range(n):
                blocks.append(_TVBottleneck(cin, 64 * 2 ** i, 2 if (j == 0 and i > 0) else 1))
                cin = 64 * 2 ** i * 4
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def test_torchvision_resnet_trunk_gets_the_linked_path():
    nat = _check_same(TVResNet(), lambda: torch.randn(2, 3, 64, 64))
    assert type(nat) is TVResNet and getattr(nat, "_tb_nativized", False)
    blocks = [b for b in nat.modules() if isinstance(b, _TVBottleneck)]
    assert len(blocks) == 4 and all(getattr(b, "_tb_kind", None) == "bottleneck" for b in blocks)
