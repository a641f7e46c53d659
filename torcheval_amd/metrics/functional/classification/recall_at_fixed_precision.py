"""Recall at fixed precision, functional API (parity: recall_at_fixed_precision.py:24-156)."""

from typing import List, Tuple

import torch

from torcheval_amd.metrics.functional.classification.precision_recall_curve import (
    _binary_precision_recall_curve_compute,
    _binary_precision_recall_curve_update_input_check,
    _multilabel_precision_recall_curve_compute,
    _multilabel_precision_recall_curve_update_input_check,
)


@torch.inference_mode()
def binary_recall_at_fixed_precision(
    input: torch.Tensor, target: torch.Tensor, *, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    """(max recall with precision >= ``min_precision``, its threshold).
    Class version: ``BinaryRecallAtFixedPrecision``."""
    _binary_recall_at_fixed_precision_update_input_check(input, target, min_precision)
    return _binary_recall_at_fixed_precision_compute(input, target, min_precision)


def _binary_recall_at_fixed_precision_update_input_check(
    input: torch.Tensor, target: torch.Tensor, min_precision: float
) -> None:
    _binary_precision_recall_curve_update_input_check(input, target)
    if not isinstance(min_precision, float) or not 0 <= min_precision <= 1:
        raise ValueError(
            f"Expected min_precision to be a float in the [0, 1] range but got {min_precision}."
        )


def _binary_recall_at_fixed_precision_compute(
    input: torch.Tensor, target: torch.Tensor, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    precision, recall, threshold = _binary_precision_recall_curve_compute(input, target)
    return _recall_at_precision(precision, recall, threshold, min_precision)


@torch.inference_mode()
def multilabel_recall_at_fixed_precision(
    input: torch.Tensor, target: torch.Tensor, *, num_labels: int, min_precision: float
) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
    """Per-label (max recall, threshold) lists.  Class: ``MultilabelRecallAtFixedPrecision``."""
    if num_labels is None and input.ndim == 2:
        num_labels = input.shape[1]
    _multilabel_recall_at_fixed_precision_update_input_check(input, target, num_labels, min_precision)
    return _multilabel_recall_at_fixed_precision_compute(input, target, num_labels, min_precision)


def _multilabel_recall_at_fixed_precision_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_labels: int, min_precision: float
) -> None:
    _multilabel_precision_recall_curve_update_input_check(input, target, num_labels)
    if not isinstance(min_precision, float) or not 0 <= min_precision <= 1:
        raise ValueError(
            f"Expected min_precision to be a float in the [0, 1] range but got {min_precision}."
        )


def _recall_at_precision(
    precision: torch.Tensor, recall: torch.Tensor, thresholds: torch.Tensor, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    max_recall = torch.max(recall[precision >= min_precision])
    thresholds = torch.cat((thresholds, thresholds.new_tensor([-1.0])))
    best_threshold = torch.max(thresholds[recall == max_recall])
    return max_recall, torch.abs(best_threshold)


def _multilabel_recall_at_fixed_precision_compute(
    input: torch.Tensor, target: torch.Tensor, num_labels: int, min_precision: float
) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
    precision, recall, thresholds = _multilabel_precision_recall_curve_compute(input, target, num_labels)
    max_recall, best_threshold = [], []
    for p, r, t in zip(precision, recall, thresholds):
        mr, bt = _recall_at_precision(p, r, t, min_precision)
        max_recall.append(mr)
        best_threshold.append(bt)
    return max_recall, best_threshold
