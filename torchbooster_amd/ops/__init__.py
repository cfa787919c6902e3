"""Hand-written gfx950 HIP ops (csrc/*.hip) with PyTorch reference fallbacks for CPU tensors."""
from torchbooster_amd.ops._ext import available, native
from torchbooster_amd.ops.norm import BatchNormAct2d, BatchNormAct1d, batch_norm_act
from torchbooster_amd.ops.loss import cross_entropy, cross_entropy_accuracy
from torchbooster_amd.ops.optim import FusedAdamW, FusedSGD, clip_grad_norm_
