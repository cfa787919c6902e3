"""Model zoo for the reference's example workloads and the north-star configs."""
from torchbooster_amd.models.resnet import (ResNet, resnet18, resnet34, resnet50, resnet101, resnet152)
