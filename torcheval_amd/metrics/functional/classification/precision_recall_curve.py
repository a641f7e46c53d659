"""Precision-recall curves, functional API (parity: precision_recall_curve.py:19-333).

Curves are variable length (one point per distinct threshold).  ROCm tensors run K3c
(csrc/kernels/curves.hip via ``ops/curves.py``): one batched payload sort over all rows, count
+ scan, one host read of the per-row sizes, emission straight into the exact outputs.  Other
devices take the vectorised ATen form in ``_curve.pr_curves`` (all rows at once, one size
read).  The reference's per-label Python loop of TorchScript calls (:296-310) and its per-row
``torch.isnan(recall[0])`` host read (:226) have no counterpart here.
"""

from typing import List, Optional, Tuple

import torch

from torcheval_amd.metrics.functional.tensor_utils import _require_samples

from torcheval_amd.metrics.functional.classification._curve import pr_curves
from torcheval_amd.ops import use_native


@torch.inference_mode()
def binary_precision_recall_curve(
    input: torch.Tensor, target: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(precision, recall, thresholds) for ``[n]`` scores; ascending thresholds with the final
    (1, 0) point appended.  Class version: ``BinaryPrecisionRecallCurve``."""
    _binary_precision_recall_curve_update(input, target)
    _require_samples(input.numel(), "binary_precision_recall_curve")
    return _binary_precision_recall_curve_compute(input, target)


def _binary_precision_recall_curve_update(input: torch.Tensor, target: torch.Tensor) -> None:
    _binary_precision_recall_curve_update_input_check(input, target)


def _binary_precision_recall_curve_compute(
    input: torch.Tensor, target: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    return _compute_for_each_class(input, target, 1)


def _binary_precision_recall_curve_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.ndim != 1:
        raise ValueError(f"input should be a one-dimensional tensor, got shape {input.shape}.")
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same shape, "
            f"got shapes {input.shape} and {target.shape}."
        )


@torch.inference_mode()
def multiclass_precision_recall_curve(
    input: torch.Tensor, target: torch.Tensor, *, num_classes: Optional[int] = None
) -> Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]:
    """One-vs-rest PR curves (lists over classes).  Class: ``MulticlassPrecisionRecallCurve``."""
    if num_classes is None and input.ndim == 2:
        num_classes = input.shape[1]
    _multiclass_precision_recall_curve_update(input, target, num_classes)
    return _multiclass_precision_recall_curve_compute(input, target, num_classes)


def _multiclass_precision_recall_curve_update(
    input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]
) -> None:
    _multiclass_precision_recall_curve_update_input_check(input, target, num_classes)


def _multiclass_precision_recall_curve_compute(
    input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]
) -> Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]:
    if num_classes is None:
        num_classes = input.shape[1]
    if use_native(input) and target.is_cuda and input.shape[0] > 0:
        from torcheval_amd.ops.curves import multiclass_pr_curves

        return multiclass_pr_curves(input, target)
    onehot = target[None, :] == torch.arange(num_classes, device=target.device)[:, None]
    return pr_curves(input.t(), onehot)


def _multiclass_precision_recall_curve_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]
) -> None:
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
    if not (input.ndim == 2 and (num_classes is None or input.shape[1] == num_classes)):
        raise ValueError(
            f"input should have shape of (num_sample, num_classes), got {input.shape} and num_classes={num_classes}."
        )


def _compute_for_each_class(
    input: torch.Tensor, target: torch.Tensor, pos_label: int
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if use_native(input) and target.is_cuda and input.numel() > 0:
        from torcheval_amd.ops.curves import binary_pr_curve

        return binary_pr_curve(input, target, pos_label)
    p, r, t = pr_curves(input.unsqueeze(0), (target == pos_label).unsqueeze(0))
    return p[0], r[0], t[0]


@torch.inference_mode()
def multilabel_precision_recall_curve(
    input: torch.Tensor, target: torch.Tensor, *, num_labels: Optional[int] = None
) -> Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]:
    """Per-label PR curves of ``[n, L]`` data.  Class: ``MultilabelPrecisionRecallCurve``."""
    if input.ndim != 2:
        raise ValueError(f"input should be a two-dimensional tensor, got shape {input.shape}.")
    if num_labels is None:
        num_labels = input.shape[1]
    _multilabel_precision_recall_curve_update(input, target, num_labels)
    return _multilabel_precision_recall_curve_compute(input, target, num_labels)


def _multilabel_precision_recall_curve_update(
    input: torch.Tensor, target: torch.Tensor, num_labels: int
) -> None:
    _multilabel_precision_recall_curve_update_input_check(input, target, num_labels)


def _multilabel_precision_recall_curve_compute(
    input: torch.Tensor, target: torch.Tensor, num_labels: int
) -> Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]:
    if use_native(input) and target.is_cuda and input.shape[0] > 0:
        from torcheval_amd.ops.curves import multilabel_pr_curves

        return multilabel_pr_curves(input, target)
    return pr_curves(input.t(), target.t() == 1)


def _multilabel_precision_recall_curve_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_labels: int
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "Expected both input.shape and target.shape to have the same shape"
            f" but got {input.shape} and {target.shape}."
        )
    if input.ndim != 2:
        raise ValueError(f"input should be a two-dimensional tensor, got shape {input.shape}.")
    if input.shape[1] != num_labels:
        raise ValueError(
            f"input should have shape of (num_sample, num_labels), got {input.shape} and num_labels={num_labels}."
        )
