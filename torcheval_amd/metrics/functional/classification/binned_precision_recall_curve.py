"""Binned precision-recall curves, functional API
(parity: functional/classification/binned_precision_recall_curve.py:20-548).

All variants run the K4 histogram kernel (ROCm) or its ATen equivalent: O(T*C) memory for
both ``optimization`` modes (the reference's "vectorized" mode materialises a [T, N, C]
bool tensor).  ``optimization`` is still validated and accepted.
"""

from typing import List, Optional, Tuple, Union

import torch

from torcheval_amd.metrics.functional.classification.precision_recall_curve import (
    _binary_precision_recall_curve_update_input_check,
    _multiclass_precision_recall_curve_update_input_check,
    _multilabel_precision_recall_curve_update_input_check,
)
from torcheval_amd.metrics.functional.tensor_utils import _threshold_check, _create_threshold_tensor
from torcheval_amd.ops.binned import binned_counts, binned_curve, binned_finalize_supported


@torch.inference_mode()
def binary_binned_precision_recall_curve(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: Union[int, List[float], torch.Tensor] = 100,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(precision, recall, thresholds) at fixed thresholds.
    Class version: ``BinaryBinnedPrecisionRecallCurve``."""
    threshold = _create_threshold_tensor(threshold, target.device)
    _binned_precision_recall_curve_param_check(threshold)
    num_tp, num_fp, num_fn = _binary_binned_precision_recall_curve_update(input, target, threshold)
    return _binary_binned_precision_recall_curve_compute(num_tp, num_fp, num_fn, threshold)


def _binary_binned_precision_recall_curve_update(
    input: torch.Tensor, target: torch.Tensor, threshold: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _binary_precision_recall_curve_update_input_check(input, target)
    return _update(input, target, threshold)


def _update(
    input: torch.Tensor, target: torch.Tensor, threshold: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    tp, fp, fn = binned_counts(input[:, None], target[:, None], threshold, 0)
    return tp[:, 0], fp[:, 0], fn[:, 0]


def _binary_binned_precision_recall_curve_compute(
    num_tp: torch.Tensor, num_fp: torch.Tensor, num_fn: torch.Tensor, threshold: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if num_tp.dim() == 1 and binned_finalize_supported(num_tp[:, None], num_fp[:, None], num_fn[:, None]):
        prec, rec = binned_curve(num_tp[:, None], num_fp[:, None], num_fn[:, None])
        return prec[0], rec[0], threshold
    precision = torch.nan_to_num(num_tp / (num_tp + num_fp), 1.0)
    recall = num_tp / (num_tp + num_fn)
    precision = torch.cat([precision, precision.new_ones(1)], dim=0)
    recall = torch.cat([recall, recall.new_zeros(1)], dim=0)
    return precision, recall, threshold


@torch.inference_mode()
def multiclass_binned_precision_recall_curve(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int] = None,
    threshold: Union[int, List[float], torch.Tensor] = 100,
    optimization: str = "vectorized",
) -> Tuple[List[torch.Tensor], List[torch.Tensor], torch.Tensor]:
    """One-vs-rest binned PR curves.  Class: ``MulticlassBinnedPrecisionRecallCurve``."""
    _optimization_param_check(optimization)
    threshold = _create_threshold_tensor(threshold, target.device)
    _binned_precision_recall_curve_param_check(threshold)
    if num_classes is None and input.ndim == 2:
        num_classes = input.shape[1]
    num_tp, num_fp, num_fn = _multiclass_binned_precision_recall_curve_update(
        input, target, num_classes, threshold, optimization
    )
    return _multiclass_binned_precision_recall_curve_compute(num_tp, num_fp, num_fn, num_classes, threshold)


def _multiclass_binned_precision_recall_curve_update(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int],
    threshold: torch.Tensor,
    optimization: str = "vectorized",
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _optimization_param_check(optimization)
    _multiclass_precision_recall_curve_update_input_check(input, target, num_classes)
    return binned_counts(input, target, threshold, 1)


def _multiclass_binned_precision_recall_curve_compute(
    num_tp: torch.Tensor,
    num_fp: torch.Tensor,
    num_fn: torch.Tensor,
    num_classes: Optional[int],
    threshold: torch.Tensor,
) -> Tuple[List[torch.Tensor], List[torch.Tensor], torch.Tensor]:
    if binned_finalize_supported(num_tp, num_fp, num_fn):
        prec, rec = binned_curve(num_tp, num_fp, num_fn)
        return list(prec), list(rec), threshold
    precision = torch.nan_to_num(num_tp / (num_tp + num_fp), 1.0)
    recall = num_tp / (num_tp + num_fn)
    precision = torch.cat([precision, precision.new_ones(1, num_classes)], dim=0)
    recall = torch.cat([recall, recall.new_zeros(1, num_classes)], dim=0)
    return list(precision.T), list(recall.T), threshold


@torch.inference_mode()
def multilabel_binned_precision_recall_curve(
    input: torch.Tensor,
    target: torch.Tensor,
    num_labels: Optional[int] = None,
    threshold: Union[int, List[float], torch.Tensor] = 100,
    optimization: str = "vectorized",
) -> Tuple[List[torch.Tensor], List[torch.Tensor], torch.Tensor]:
    """Per-label binned PR curves.  Class: ``MultilabelBinnedPrecisionRecallCurve``."""
    _optimization_param_check(optimization)
    threshold = _create_threshold_tensor(threshold, target.device)
    _binned_precision_recall_curve_param_check(threshold)
    if input.ndim != 2:
        raise ValueError(f"input should be a two-dimensional tensor, got shape {input.shape}.")
    if num_labels is None:
        num_labels = input.shape[1]
    num_tp, num_fp, num_fn = _multilabel_binned_precision_recall_curve_update(
        input, target, num_labels, threshold, optimization
    )
    return _multilabel_binned_precision_recall_curve_compute(num_tp, num_fp, num_fn, num_labels, threshold)


def _multilabel_binned_precision_recall_curve_update(
    input: torch.Tensor,
    target: torch.Tensor,
    num_labels: int,
    threshold: torch.Tensor,
    optimization: str = "vectorized",
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _optimization_param_check(optimization)
    _multilabel_precision_recall_curve_update_input_check(input, target, num_labels)
    return binned_counts(input, target, threshold, 0)


def _multilabel_binned_precision_recall_curve_compute(
    num_tp: torch.Tensor,
    num_fp: torch.Tensor,
    num_fn: torch.Tensor,
    num_labels: int,
    threshold: torch.Tensor,
) -> Tuple[List[torch.Tensor], List[torch.Tensor], torch.Tensor]:
    return _multiclass_binned_precision_recall_curve_compute(num_tp, num_fp, num_fn, num_labels, threshold)


def _binned_precision_recall_curve_param_check(threshold: torch.Tensor) -> None:
    _threshold_check(threshold)


def _optimization_param_check(optimization: str) -> None:
    if optimization not in ("vectorized", "memory"):
        raise ValueError(
            f"Unknown memory approach: expected 'vectorized' or 'memory', but got {optimization}."
        )
