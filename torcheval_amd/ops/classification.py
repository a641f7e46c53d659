"""Python wrappers of the K1 classification-count kernels (csrc/kernels/classification.hip).

All wrappers accumulate INTO caller-provided float32 tensors (metric states or fresh zero
buffers), so a class-metric ``update()`` is exactly one kernel launch.
"""

from typing import Optional

import torch

from torcheval_amd.ops import MAX_BLOCKS, native

_SCORE_DTYPES = (torch.float32, torch.bfloat16, torch.float16)
_LABEL_DTYPES = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)


def cls_counts_supported(input: torch.Tensor, target: torch.Tensor) -> bool:
    """Whether the fused kernel handles this (input, target) dtype/shape combination."""
    if target.dtype not in _LABEL_DTYPES or target.dim() != 1:
        return False
    if input.dim() == 2:
        return input.dtype in _SCORE_DTYPES
    if input.dim() == 1:
        return input.dtype in _LABEL_DTYPES
    return False


def cls_counts(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    k: int = 1,
    num_classes: int = 0,
    micro_correct: Optional[torch.Tensor] = None,
    micro_total: Optional[torch.Tensor] = None,
    cls_correct: Optional[torch.Tensor] = None,
    cls_label: Optional[torch.Tensor] = None,
    cls_pred: Optional[torch.Tensor] = None,
    confusion: Optional[torch.Tensor] = None,
    err: Optional[torch.Tensor] = None,
) -> None:
    """Accumulate argmax / top-k correctness counts and class histograms in one pass."""
    if not target.is_contiguous():
        target = target.contiguous()
    native().cls_counts(
        input,
        target,
        int(k),
        int(num_classes),
        micro_correct,
        micro_total,
        cls_correct,
        cls_label,
        cls_pred,
        confusion,
        err,
        MAX_BLOCKS,
    )


def binary_counts(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: float = 0.5,
    weight: Optional[torch.Tensor] = None,
    tp: Optional[torch.Tensor] = None,
    fp: Optional[torch.Tensor] = None,
    tn: Optional[torch.Tensor] = None,
    fn: Optional[torch.Tensor] = None,
    total: Optional[torch.Tensor] = None,
    strict: bool = False,
) -> None:
    """Accumulate thresholded binary confusion counts (tp, fp, tn, fn) in one pass."""
    native().binary_counts(
        input, target, weight, float(threshold), tp, fp, tn, fn, total, int(strict), MAX_BLOCKS
    )
