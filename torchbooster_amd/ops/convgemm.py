"""Convolutions as native im2col / col2im + the native GEMM engine.

For the conv shapes the implicit-GEMM kernels handle poorly -- 3-channel image
layers with 9x9 / 4x4 windows (StyleNet input, reference online.py:57; DCGAN
discriminator input / generator output) and 512-channel convs over a few hundred
pixels (VGG-19 at batch 1, offline.py:104) -- the routing tables used to keep
MIOpen.  These functions give every such direction a native candidate
(csrc/im2col.hip + csrc/gemm.hip / gemm8.hip); ``ops.conv._route`` times it
against the others, and ``TBAMD_CONV_NO_MIOPEN=1`` removes MIOpen from the
candidates altogether.

Layouts: activations NHWC (channels_last NCHW views), conv weights [K, C, R, S]
channels_last (= [K][R][S][C] memory: the im2col k order), transposed-conv
weights [Cin, Cout, R, S].
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from torchbooster_amd.ops import gemm as G
from torchbooster_amd.ops._ext import native

__all__ = ["supported", "conv_fwd", "conv_wgrad", "conv_dgrad", "convT_fwd", "convT_wgrad", "out_size"]


def supported(x: Tensor, w: Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and w.dim() == 4)


def out_size(h: int, r: int, stride: int, pad: int, up: int = 1) -> int:
    return (h * up + 2 * pad - r) // stride + 1


def _nhwc(x: Tensor) -> Tensor:
    return x.contiguous(memory_format=torch.channels_last)


def _kp(n: int) -> int:
    return (n + 7) // 8 * 8


def _w_rows(w: Tensor) -> Tensor:
    """[K, C, R, S] -> [K, KP] in (r, s, c) order, zero tail to a multiple of 8."""
    K = w.shape[0]
    rows = w.permute(0, 2, 3, 1).reshape(K, -1)
    kp = _kp(rows.shape[1])
    if kp != rows.shape[1]:
        rows = torch.nn.functional.pad(rows, (0, kp - rows.shape[1]))
    return rows.contiguous()


def _nhwc_out(rows: Tensor, N: int, P: int, Q: int, K: int) -> Tensor:
    return rows.view(N, P, Q, K).permute(0, 3, 1, 2)  # channels_last view


def conv_fwd(x: Tensor, w: Tensor, bias: Optional[Tensor], stride: int, pad: int, up: int = 1,
             reflect: bool = False, relu: bool = False) -> Tensor:
    """conv2d(pad(upsample(x)), w) + bias [-> ReLU], NHWC out."""
    N, C, H, W = x.shape
    K, _, R, S = w.shape
    P, Q = out_size(H, R, stride, pad, up), out_size(W, S, stride, pad, up)
    col = native().im2col(_nhwc(x), R, S, P, Q, stride, pad, up, reflect)
    y = G.mm_nt(col, _w_rows(w), bias=bias, relu=relu, blas=False)
    return _nhwc_out(y, N, P, Q, K)


def conv_wgrad(dy: Tensor, x: Tensor, w_shape, stride: int, pad: int, up: int = 1, reflect: bool = False) -> Tensor:
    """dW = dYᵀ im2col(x) -> [K, C, R, S] channels_last."""
    N, C, H, W = x.shape
    K, _, R, S = w_shape
    P, Q = dy.shape[2], dy.shape[3]
    col = native().im2col(_nhwc(x), R, S, P, Q, stride, pad, up, reflect)
    dyr = _nhwc(dy).permute(0, 2, 3, 1).reshape(N * P * Q, K)
    dw = G.mm_tn(dyr, col)[:, : R * S * C]  # [K, RSC]
    return dw.reshape(K, R, S, C).permute(0, 3, 1, 2)


def conv_dgrad(dy: Tensor, w: Tensor, x_shape, stride: int, pad: int) -> Tensor:
    """dX = col2im(dY W) (zero padding, no upsampling)."""
    N, C, H, W = x_shape
    K, _, R, S = w.shape
    P, Q = dy.shape[2], dy.shape[3]
    dyr = _nhwc(dy).permute(0, 2, 3, 1).reshape(N * P * Q, K)
    wr = _w_rows(w)  # [K, KP]
    dcol = G.mm_nn(dyr, wr)  # [NPQ, KP]
    return native().col2im(dcol.contiguous(), N, C, H, W, R, S, P, Q, stride, pad)


def _wT_rows(w: Tensor) -> Tensor:
    """transposed-conv weight [Cin, Cout, R, S] -> [KP(r, s, co), Cin] rows."""
    Cin, Cout, R, S = w.shape
    rows = w.permute(2, 3, 1, 0).reshape(R * S * Cout, Cin)
    kp = _kp(rows.shape[0])
    if kp != rows.shape[0]:
        rows = torch.cat([rows, rows.new_zeros(kp - rows.shape[0], Cin)], 0)
    return rows.contiguous()


def convT_fwd(x: Tensor, w: Tensor, bias: Optional[Tensor], stride: int, pad: int) -> Tensor:
    """conv_transpose2d(x, w) = col2im(x Wᵀ): the input gradient of conv(Cout -> Cin)."""
    N, Cin, Hi, Wi = x.shape
    _, Cout, R, S = w.shape
    Ho, Wo = (Hi - 1) * stride - 2 * pad + R, (Wi - 1) * stride - 2 * pad + S
    xr = _nhwc(x).permute(0, 2, 3, 1).reshape(N * Hi * Wi, Cin)
    cols = G.mm_nt(xr, _wT_rows(w), blas=False)  # [N Hi Wi, KP(r, s, co)]
    return native().col2im(cols.contiguous(), N, Cout, Ho, Wo, R, S, Hi, Wi, stride, pad, bias)


def convT_wgrad(x: Tensor, dy: Tensor, w_shape, stride: int, pad: int) -> Tensor:
    """dW[ci, co, r, s] = sum over input pixels x[., ci] dY[window(r, s), co] = xᵀ im2col(dY)."""
    N, Cin, Hi, Wi = x.shape
    _, Cout, R, S = w_shape
    col = native().im2col(_nhwc(dy), R, S, Hi, Wi, stride, pad, 1, False)  # [N Hi Wi, KP(r, s, co)]
    xr = _nhwc(x).permute(0, 2, 3, 1).reshape(N * Hi * Wi, Cin)
    dw = G.mm_tn(xr, col)[:, : R * S * Cout]  # [Cin, RSCout]
    return dw.reshape(Cin, R, S, Cout).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
