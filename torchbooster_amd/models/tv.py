"""torchvision-layout models built from stock ``torch.nn`` modules, and pretrained-weight loading.

The reference fine-tunes ``torchvision.models.resnet18(pretrained=True)``
(/root/reference/examples/img_cls/resnet/resnet.py:111-112) and computes its
style losses on frozen pretrained VGG features (offline.py:104, online.py:166,
adain.py:179).  torchvision is not part of this stack and there is no network,
so:

* :class:`ResNet` / :func:`resnet18` ... :func:`resnet152` reproduce
  torchvision's module tree exactly (``conv1``, ``bn1``, ``relu``, ``maxpool``,
  ``layer1``-``layer4`` of ``BasicBlock`` / ``Bottleneck`` with
  ``downsample = Sequential(conv1x1, bn)``, ``avgpool``, ``fc``), so a
  torchvision state dict loads with ``strict=True``.  They are plain stock
  modules: :func:`~torchbooster_amd.nativize.nativize` (applied by
  ``EnvironementConfig.make``) puts them on the native kernels with the same
  fusions as the hand-wired :mod:`~torchbooster_amd.models.resnet`.
* :func:`load_weights` reads a local torchvision-layout checkpoint with
  ``torch.load(weights_only=True)`` (executes nothing from the file) into any
  of these models or into :class:`~torchbooster_amd.models.vgg.VGG` (whose
  ``features`` / ``classifier`` indices are torchvision's).
"""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, List, Optional, Sequence, Type, Union

import torch
from torch import Tensor, nn

__all__ = ["BasicBlock", "Bottleneck", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "load_weights", "extract_state_dict"]

_LOG = logging.getLogger(__name__)


def _conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride, 1, bias=False)


def _conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = _conv3x3(cin, width, stride)
        self.bn1 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(width, width)
        self.bn2 = nn.BatchNorm2d(width)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: Tensor) -> Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class Bottleneck(nn.Module):
    """v1.5 bottleneck (stride on the 3x3), torchvision's layout and names."""

    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = _conv1x1(cin, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv1x1(width, width * self.expansion)
        self.bn3 = nn.BatchNorm2d(width * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: Tensor) -> Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, block: Union[Type[BasicBlock], Type[Bottleneck]], layers: Sequence[int],
                 num_classes: int = 1000, zero_init_residual: bool = False) -> None:
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], 2)
        self.layer3 = self._make_layer(block, 256, layers[2], 2)
        self.layer4 = self._make_layer(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, width: int, n: int, stride: int = 1) -> nn.Sequential:
        down = None
        if stride != 1 or self.inplanes != width * block.expansion:
            down = nn.Sequential(_conv1x1(self.inplanes, width * block.expansion, stride),
                                 nn.BatchNorm2d(width * block.expansion))
        layers: List[nn.Module] = [block(self.inplanes, width, stride, down)]
        self.inplanes = width * block.expansion
        for _ in range(1, n):
            layers.append(block(self.inplanes, width))
        return nn.Sequential(*layers)

    def forward(self, x: Tensor) -> Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(num_classes: int = 1000, weights: Optional[str] = None, **kw) -> ResNet:
    return _build(BasicBlock, [2, 2, 2, 2], num_classes, weights, **kw)


def resnet34(num_classes: int = 1000, weights: Optional[str] = None, **kw) -> ResNet:
    return _build(BasicBlock, [3, 4, 6, 3], num_classes, weights, **kw)


def resnet50(num_classes: int = 1000, weights: Optional[str] = None, **kw) -> ResNet:
    return _build(Bottleneck, [3, 4, 6, 3], num_classes, weights, **kw)


def resnet101(num_classes: int = 1000, weights: Optional[str] = None, **kw) -> ResNet:
    return _build(Bottleneck, [3, 4, 23, 3], num_classes, weights, **kw)


def resnet152(num_classes: int = 1000, weights: Optional[str] = None, **kw) -> ResNet:
    return _build(Bottleneck, [3, 8, 36, 3], num_classes, weights, **kw)


def _build(block, layers, num_classes, weights, **kw) -> ResNet:
    m = ResNet(block, layers, num_classes, **kw)
    if weights:
        load_weights(m, weights, strict=False)
    return m


def extract_state_dict(obj: Any) -> Dict[str, Tensor]:
    """The tensor dict inside a checkpoint: a bare state dict, or one nested under
    ``state_dict`` / ``model`` (SaveCallback files); ``module.`` prefixes stripped."""
    if isinstance(obj, dict):
        for key in ("state_dict", "model"):
            if key in obj and isinstance(obj[key], dict):
                return extract_state_dict(obj[key])
    if not isinstance(obj, dict) or not all(isinstance(v, Tensor) for v in obj.values()):
        raise ValueError("checkpoint does not hold a state dict of tensors")
    return {(k[7:] if k.startswith("module.") else k): v for k, v in obj.items()}


def load_weights(model: nn.Module, path: Union[str, os.PathLike], strict: bool = True) -> nn.Module:
    """Load a torchvision-layout checkpoint from a LOCAL file into ``model``.

    ``torch.load(..., weights_only=True)``: nothing in the file is executed.  With
    ``strict=False`` keys whose shape does not match (e.g. a 1000-class ``fc`` into
    a 10-class head: the reference's fine-tune, resnet.py:111-112) are skipped and
    reported, like torchvision's ``pretrained`` + head replacement."""
    sd = extract_state_dict(torch.load(os.fspath(path), map_location="cpu", weights_only=True))
    own = model.state_dict()
    if not strict:
        skipped = [k for k, v in sd.items() if k in own and own[k].shape != v.shape]
        sd = {k: v for k, v in sd.items() if k not in skipped}
        if skipped:
            _LOG.warning("load_weights: shape mismatch, kept the model's own %s", skipped)
    res = model.load_state_dict(sd, strict=strict)
    if not strict and (res.missing_keys or res.unexpected_keys):
        _LOG.warning("load_weights: missing %s, unexpected %s", res.missing_keys, res.unexpected_keys)
    return model
