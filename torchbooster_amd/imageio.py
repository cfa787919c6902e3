"""Image input/output for the examples (what the reference gets from torchvision / PIL).

The reference examples load their style / content images with PIL and
torchvision transforms (/root/reference/examples/img_stt/offline/offline.py:108-119,
online.py:168-176, adain.py:163-179), and show results with ``make_grid`` +
``ToPILImage`` (online.py:160-162,190, gan.py:131, vae.py:135).  torchvision is
not part of this stack; these helpers cover exactly those uses with PIL + torch:

* :func:`load_image` -- ``Resize(size)`` (shorter side) + ``CenterCrop(size)`` +
  ``ToTensor`` of a LOCAL file -> ``[1, 3, H, W]`` float in [0, 1];
* :func:`normalize` / :func:`denormalize` -- the ImageNet ``Normalize`` pair;
* :func:`make_grid` -- batch -> one padded grid image;
* :func:`save_image` -- tensor -> PNG (optionally min-max stretched, the
  reference's ``hdr`` lambda), creating the parent directory.
"""
from __future__ import annotations

import logging
import os
from typing import Optional, Sequence, Union

import torch
from torch import Tensor

__all__ = ["IMAGENET_MEAN", "IMAGENET_STD", "load_image", "normalize", "denormalize", "make_grid", "save_image",
           "image_or_synthetic"]

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
_LOG = logging.getLogger(__name__)


def load_image(path: Union[str, os.PathLike], size: Optional[int] = None, crop: bool = True) -> Tensor:
    """RGB image from a local file as ``[1, 3, H, W]`` float32 in [0, 1]; ``size``
    resizes the shorter side (bilinear) and, with ``crop``, center-crops to a square."""
    from PIL import Image

    import numpy as np

    img = Image.open(os.fspath(path)).convert("RGB")
    if size is not None:
        w, h = img.size
        s = size / min(w, h)
        img = img.resize((max(size, round(w * s)), max(size, round(h * s))), Image.BILINEAR)
        if crop:
            w, h = img.size
            l, t = (w - size) // 2, (h - size) // 2
            img = img.crop((l, t, l + size, t + size))
    a = np.asarray(img, dtype=np.uint8).copy()
    return torch.from_numpy(a).permute(2, 0, 1).unsqueeze(0).float().div_(255.0)


def _stats(x: Tensor, mean: Sequence[float], std: Sequence[float]):
    m = torch.tensor(mean, dtype=x.dtype, device=x.device).view(1, -1, 1, 1)
    s = torch.tensor(std, dtype=x.dtype, device=x.device).view(1, -1, 1, 1)
    return m, s


def normalize(x: Tensor, mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD) -> Tensor:
    m, s = _stats(x, mean, std)
    return (x - m) / s


def denormalize(x: Tensor, mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD) -> Tensor:
    m, s = _stats(x, mean, std)
    return x * s + m


def make_grid(x: Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> Tensor:
    """``[B, C, H, W]`` -> ``[C, rows*(H+p)+p, nrow*(W+p)+p]`` (torchvision's layout)."""
    x = x.detach()
    if x.dim() == 3:
        x = x.unsqueeze(0)
    B, C, H, W = x.shape
    ncol = min(nrow, B)
    nr = (B + ncol - 1) // ncol
    grid = x.new_full((C, nr * (H + padding) + padding, ncol * (W + padding) + padding), pad_value)
    for i in range(B):
        r, c = divmod(i, ncol)
        y0, x0 = r * (H + padding) + padding, c * (W + padding) + padding
        grid[:, y0:y0 + H, x0:x0 + W] = x[i]
    return grid


def save_image(x: Tensor, path: Union[str, os.PathLike], stretch: bool = False, nrow: int = 8) -> str:
    """Write ``x`` ([C, H, W] or a [B, C, H, W] batch, made a grid) as a PNG.  ``stretch``:
    min-max to [0, 1] first (the reference's ``hdr`` display lambda); else clamp."""
    from PIL import Image

    x = x.detach().float().cpu()
    if x.dim() == 4:
        x = make_grid(x, nrow=nrow) if x.shape[0] > 1 else x[0]
    if stretch:
        lo, hi = x.min(), x.max()
        x = (x - lo) / (hi - lo + 1e-12)
    x = x.clamp(0, 1)
    if x.shape[0] == 1:
        x = x.expand(3, -1, -1)
    a = (x.permute(1, 2, 0) * 255.0 + 0.5).to(torch.uint8).numpy()
    path = os.fspath(path)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    Image.fromarray(a).save(path)
    return path


def image_or_synthetic(path: str, size: int, what: str, generator: Optional[torch.Generator] = None) -> Tensor:
    """:func:`load_image` of ``path`` when set, else a uniform-noise image with a warning
    (there is no network here for the reference's image URLs)."""
    if path:
        return load_image(path, size)
    _LOG.warning("no %s image path configured: using a synthetic %dx%d image", what, size, size)
    return torch.rand(1, 3, size, size, generator=generator)
