"""Fused softmax cross-entropy (+ label smoothing) with batch accuracy.

Reference call sites: ``cross_entropy(logits, labels, label_smoothing=...)``
followed by ``metrics.accuracy(logits, labels)``
(/root/reference/examples/img_cls/resnet/resnet.py:61-62,
/root/reference/torchbooster/metrics.py:11-27).  One HIP kernel computes both
(csrc/loss.hip); SURVEY.md §2.3.1 K9/K10.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch.autograd.function import once_differentiable
import torch.nn.functional as F
from torch import Tensor

from torchbooster_amd.ops._ext import native, use_native


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing, ignore_index):
        C = native()
        stats, lse = C.ce_forward(logits, labels, smoothing, ignore_index)
        ctx.save_for_backward(logits, labels, lse, stats)
        ctx.cfg = (smoothing, ignore_index)
        loss = stats[0]
        acc = stats[1]
        ctx.mark_non_differentiable(acc)
        return loss, acc

    @staticmethod
    @once_differentiable
    def backward(ctx, gloss, gacc):
        C = native()
        logits, labels, lse, stats = ctx.saved_tensors
        smoothing, ignore_index = ctx.cfg
        if gloss is None:
            return None, None, None, None
        dl = C.ce_backward(logits, labels, lse, gloss.reshape(1), stats, smoothing, ignore_index)
        return dl, None, None, None


def cross_entropy_accuracy(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0,
                           ignore_index: int = -100) -> Tuple[Tensor, Tensor]:
    """Mean cross-entropy and batch accuracy (``(argmax == label).sum() / N``)."""
    if use_native(logits) and logits.dim() == 2 and labels.dim() == 1:
        return _CEFn.apply(logits, labels, float(label_smoothing), int(ignore_index))
    loss = F.cross_entropy(logits.float(), labels, ignore_index=ignore_index, label_smoothing=label_smoothing)
    with torch.no_grad():
        acc = (logits.argmax(dim=-1) == labels).sum() / logits.size(0)
    return loss, acc


def cross_entropy(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0,
                  ignore_index: int = -100) -> Tensor:
    return cross_entropy_accuracy(logits, labels, label_smoothing, ignore_index)[0]
