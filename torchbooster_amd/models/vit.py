"""Vision Transformer (ViT-B/16 and friends) — BASELINE.json config 5.

Not part of the reference (it has no attention model); built
for the north-star "ViT-B/16 224px bf16 DDP via torchbooster.lmdb + cosine
scheduler" configuration.  Pre-norm blocks; the residual add of each sub-block
is fused into the following LayerNorm kernel (``LayerNorm(x, residual)``
returns both the normalised tensor and the updated residual stream), patch
embedding is a 16x16/s16 conv (a GEMM over non-overlapping patches).
Attention is the native flash-style MFMA kernel (ops/attention.py,
csrc/attention.hip) reading the packed QKV projection output through strides
and writing the packed dQKV gradient; no Triton / aotriton kernels are used.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops.attention import attention_packed
from torchbooster_amd.ops.conv import Conv2d

from torchbooster_amd.ops.norm import LayerNorm
from torchbooster_amd.ops.linear import GeluLink, Linear, LinearGELU, linear

__all__ = ["ViT", "vit_b_16", "vit_s_16", "vit_tiny", "Attention", "Block"]


class Attention(nn.Module):
    def __init__(self, dim: int, heads: int) -> None:
        super().__init__()
        self.heads = heads
        self.hd = dim // heads
        self.qkv = Linear(dim, 3 * dim)
        self.proj = Linear(dim, dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.proj(attention_packed(self.qkv(x), self.heads, 1.0 / math.sqrt(self.hd)))


class MLP(nn.Module):
    def __init__(self, dim: int, hidden: int) -> None:
        super().__init__()
        self.fc1 = LinearGELU(dim, hidden)  # GELU fused into its backward / bias-grad pass
        self.fc2 = Linear(hidden, dim)

    def forward(self, x: Tensor) -> Tensor:
        # fc2 is the hidden activation's only consumer: its input gradient takes fc1's GELU
        # backward and bias gradient into the same GEMM epilogue (ops/linear.py GeluLink)
        link = GeluLink()
        return self.fc2(self.fc1(x, link), gelu_in=link)


class Block(nn.Module):
    def __init__(self, dim: int, heads: int, mlp_ratio: float = 4.0) -> None:
        super().__init__()
        self.ln1 = LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.ln2 = LayerNorm(dim, eps=1e-6)
        self.mlp = MLP(dim, int(dim * mlp_ratio))

    def forward(self, x: Tensor, pending: Optional[Tensor] = None):
        """``x``: residual stream; ``pending``: a sub-block output not yet added
        to it.  Returns (stream, pending) so adds fuse into the next LayerNorm."""
        if pending is None:
            h = self.ln1(x)
        else:
            h, x = self.ln1(x, pending)
        a = self.attn(h)
        h, x = self.ln2(x, a)
        return x, self.mlp(h)


class ViT(nn.Module):
    def __init__(self, image: int = 224, patch: int = 16, dim: int = 768, depth: int = 12, heads: int = 12,
                 mlp_ratio: float = 4.0, num_classes: int = 1000, in_ch: int = 3) -> None:
        super().__init__()
        self.patch = Conv2d(in_ch, dim, patch, patch)
        n = (image // patch) ** 2
        self.cls = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos = nn.Parameter(torch.zeros(1, n + 1, dim))
        self.blocks = nn.ModuleList([Block(dim, heads, mlp_ratio) for _ in range(depth)])
        self.norm = LayerNorm(dim, eps=1e-6)
        self.head = Linear(dim, num_classes)
        nn.init.trunc_normal_(self.pos, std=0.02)
        nn.init.trunc_normal_(self.cls, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)

    def embed(self, x: Tensor) -> Tensor:
        """Patch embedding -> [B, N, D].  On the native path the non-overlapping
        16x16/s16 conv is one GEMM: a patchify copy ([B*N, C*p*p] rows in the
        conv weight's (c, kh, kw) order) and the native Linear (bias fused; its
        weight gradient is the split-K dW kernel)."""
        B, C, H, W = x.shape
        p = self.patch.kernel_size[0]
        w = self.patch.weight
        if x.is_cuda and x.dtype == torch.bfloat16 and (C * p * p) % 8 == 0 and H % p == 0 and W % p == 0:
            h, wn = H // p, W // p
            rows = x.reshape(B, C, h, p, wn, p).permute(0, 2, 4, 1, 3, 5).reshape(B * h * wn, C * p * p)
            y = linear(rows, w.reshape(w.shape[0], -1), self.patch.bias)
            return y.view(B, h * wn, -1)
        return self.patch(x).flatten(2).transpose(1, 2)

    def forward(self, x: Tensor) -> Tensor:
        x = self.embed(x)  # [B, N, D]
        x = torch.cat([self.cls.expand(x.shape[0], -1, -1).to(x.dtype), x], dim=1) + self.pos.to(x.dtype)
        pending = None
        for blk in self.blocks:
            x, pending = blk(x, pending)
        h, _ = self.norm(x, pending)
        return self.head(h[:, 0])


def vit_b_16(num_classes: int = 1000, image: int = 224) -> ViT:
    return ViT(image, 16, 768, 12, 12, 4.0, num_classes)


def vit_s_16(num_classes: int = 1000, image: int = 224) -> ViT:
    return ViT(image, 16, 384, 12, 6, 4.0, num_classes)


def vit_tiny(num_classes: int = 10, image: int = 32) -> ViT:
    return ViT(image, 4, 192, 4, 3, 4.0, num_classes)
