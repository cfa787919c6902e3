"""VGG-16 / VGG-19 feature extractors (torchvision layer indexing).

The style-transfer examples hook ``vgg19().features[i]`` / ``vgg16().features[i]``
by index (/root/reference/examples/img_stt/offline/offline.py:67-70,
offline.yml style_layers [0, 5, 10, 19, 28], content 29;
online.yml layers [3, 8, 15, 22]), so the Sequential keeps torchvision's exact
ordering: Conv2d, ReLU, ..., MaxPool2d.  Weights are random-init here (no
network); the conv hot path runs NHWC (channels_last).
"""
from __future__ import annotations

from typing import List, Union

from torch import nn

from torchbooster_amd.ops.conv import Conv2d, ConvReLUSequential
from torchbooster_amd.ops.linear import Linear
from torchbooster_amd.ops.pool import MaxPool2d

__all__ = ["VGG", "vgg16", "vgg19", "vgg_features", "CFG"]

CFG = {
    "vgg11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "vgg19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512,
              "M"],
}


def vgg_features(cfg: List[Union[int, str]], in_ch: int = 3) -> nn.Sequential:
    layers: List[nn.Module] = []
    c = in_ch
    for v in cfg:
        if v == "M":
            layers.append(MaxPool2d(2, 2))
        else:
            layers.append(Conv2d(c, int(v), 3, padding=1))
            layers.append(nn.ReLU(inplace=True))
            c = int(v)
    # conv -> ReLU pairs run as one conv with the ReLU in its epilogue (unhooked pairs only)
    return ConvReLUSequential(*layers)


class VGG(nn.Module):
    def __init__(self, cfg: str = "vgg19", num_classes: int = 1000) -> None:
        super().__init__()
        self.features = vgg_features(CFG[cfg])
        self.avgpool = nn.AdaptiveAvgPool2d((7, 7))
        self.classifier = nn.Sequential(Linear(512 * 49, 4096), nn.ReLU(True), nn.Dropout(), Linear(4096, 4096),
                                        nn.ReLU(True), nn.Dropout(), Linear(4096, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.avgpool(self.features(x)).flatten(1)
        return self.classifier(x)


def vgg16(num_classes: int = 1000) -> VGG:
    return VGG("vgg16", num_classes)


def vgg19(num_classes: int = 1000) -> VGG:
    return VGG("vgg19", num_classes)
