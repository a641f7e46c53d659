"""Binned AUPRC, functional API (parity: functional/classification/binned_auprc.py:28-470).

The per-task / per-class Python loops of the reference (binned_auprc.py:86-112, 456-470)
become one batched K4 histogram + one vectorised Riemann sum over all rows.
"""

from typing import List, Optional, Tuple, Union

import torch

from torcheval_amd.metrics.functional.classification.binned_precision_recall_curve import (
    _optimization_param_check,
)
from torcheval_amd.metrics.functional.tensor_utils import _threshold_check, _create_threshold_tensor
from torcheval_amd.ops.binned import binned_counts, binned_finalize, binned_finalize_supported

DEFAULT_NUM_THRESHOLD = 100


def _binned_riemann(tp: torch.Tensor, fp: torch.Tensor, fn: torch.Tensor) -> torch.Tensor:
    """tp/fp/fn: [T, R] -> float32 [R] Riemann AUPRC over the binned PR curves (NaN -> 0)."""
    if binned_finalize_supported(tp, fp, fn):
        return binned_finalize(tp, fp, fn, auroc=False, auprc=True)[1]
    precision = torch.nan_to_num(tp / (tp + fp), 1.0)
    recall = tp / (tp + fn)
    R = tp.shape[1]
    precision = torch.cat([precision, precision.new_ones(1, R)])
    recall = torch.cat([recall, recall.new_zeros(1, R)])
    auprc = -((recall[1:] - recall[:-1]) * precision[:-1]).sum(0)
    return torch.nan_to_num(auprc, nan=0.0)


@torch.inference_mode()
def binary_binned_auprc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_tasks: int = 1,
    threshold: Union[int, List[float], torch.Tensor] = DEFAULT_NUM_THRESHOLD,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """(AUPRC, thresholds) with scores binned at ``threshold``.  Class: ``BinaryBinnedAUPRC``."""
    threshold = _create_threshold_tensor(threshold, target.device)
    _binary_binned_auprc_param_check(num_tasks, threshold)
    _binary_binned_auprc_update_input_check(input, target, num_tasks, threshold)
    return _binary_binned_auprc_compute(input, target, num_tasks, threshold), threshold


def _binary_binned_auprc_compute(
    input: torch.Tensor, target: torch.Tensor, num_tasks: int, threshold: torch.Tensor
) -> torch.Tensor:
    x = input if input.ndim == 2 else input.unsqueeze(0)
    t = target if target.ndim == 2 else target.unsqueeze(0)
    tp, fp, fn = binned_counts(x.t(), t.t(), threshold, 0)
    auprc = _binned_riemann(tp, fp, fn)
    if num_tasks == 1 and input.ndim == 1:
        return auprc[0]
    return auprc


def _binary_binned_auprc_param_check(num_tasks: int, threshold: torch.Tensor) -> None:
    if num_tasks < 1:
        raise ValueError("`num_tasks` has to be at least 1.")
    _binned_threshold_check(threshold)


def _binned_threshold_check(threshold: torch.Tensor) -> None:
    if threshold.ndim != 1:
        raise ValueError(f"`threshold` should be 1-dimensional, but got {threshold.ndim}D tensor.")
    _threshold_check(threshold, endpoints=True)


def _binary_binned_auprc_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_tasks: int, threshold: torch.Tensor
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same shape, "
            f"got shapes {input.shape} and {target.shape}."
        )
    elif num_tasks == 1:
        if input.ndim not in (1, 2):
            raise ValueError(
                f"`num_tasks = 1`, `input` is expected to be 1D or 2D tensor, but got shape {input.shape}."
            )
    elif input.ndim != 2:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input` is expected to be 2D tensor, but got shape {input.shape}."
        )
    elif input.shape[0] != num_tasks:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input`'s shape is expected to be ({num_tasks}, num_samples), but got shape {input.shape}."
        )


@torch.inference_mode()
def multiclass_binned_auprc(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int] = None,
    *,
    threshold: Union[int, List[float], torch.Tensor] = DEFAULT_NUM_THRESHOLD,
    average: Optional[str] = "macro",
    optimization: str = "vectorized",
) -> Tuple[torch.Tensor, torch.Tensor]:
    """One-vs-rest binned AUPRC.  Class: ``MulticlassBinnedAUPRC``."""
    _optimization_param_check(optimization)
    if num_classes is None:
        num_classes = input.shape[1]
    threshold = _create_threshold_tensor(threshold, target.device)
    _multiclass_binned_auprc_param_check(num_classes, threshold, average)
    _multiclass_binned_auprc_update_input_check(input, target, num_classes)
    return (
        _multiclass_binned_auprc_compute(input, target, num_classes, threshold, average, optimization),
        threshold,
    )


def _multiclass_binned_auprc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: int,
    threshold: torch.Tensor,
    average: Optional[str] = "macro",
    optimization: str = "vectorized",
) -> torch.Tensor:
    tp, fp, fn = binned_counts(input, target, threshold, 1)
    return _average(_binned_riemann(tp, fp, fn), average)


def _average(auprcs: torch.Tensor, average: Optional[str]) -> torch.Tensor:
    return torch.mean(auprcs) if average == "macro" else auprcs


def _multiclass_binned_auprc_param_check(
    num_classes: int, threshold: torch.Tensor, average: Optional[str]
) -> None:
    average_options = ("macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if num_classes < 2:
        raise ValueError("`num_classes` has to be at least 2.")
    _binned_threshold_check(threshold)


def _multiclass_binned_auprc_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_classes: int
) -> None:
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
    if not (input.ndim == 2 and input.shape[1] == num_classes):
        raise ValueError(
            f"input should have shape of (num_sample, num_classes), got {input.shape} and num_classes={num_classes}."
        )


@torch.inference_mode()
def multilabel_binned_auprc(
    input: torch.Tensor,
    target: torch.Tensor,
    num_labels: Optional[int] = None,
    *,
    threshold: Union[int, List[float], torch.Tensor] = DEFAULT_NUM_THRESHOLD,
    average: Optional[str] = "macro",
    optimization: str = "vectorized",
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-label binned AUPRC.  Class: ``MultilabelBinnedAUPRC``."""
    _optimization_param_check(optimization)
    if num_labels is None:
        num_labels = input.shape[1]
    threshold = _create_threshold_tensor(threshold, target.device)
    _multilabel_binned_auprc_param_check(num_labels, threshold, average)
    _multilabel_binned_auprc_update_input_check(input, target, num_labels)
    return (
        _multilabel_binned_auprc_compute(input, target, num_labels, threshold, average, optimization),
        threshold,
    )


def _multilabel_binned_auprc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    num_labels: int,
    threshold: torch.Tensor,
    average: Optional[str] = "macro",
    optimization: str = "vectorized",
) -> torch.Tensor:
    tp, fp, fn = binned_counts(input, target, threshold, 0)
    return _average(_binned_riemann(tp, fp, fn), average)


def _multilabel_binned_auprc_param_check(
    num_labels: int, threshold: torch.Tensor, average: Optional[str]
) -> None:
    average_options = ("macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if num_labels < 2:
        raise ValueError("`num_labels` has to be at least 2.")
    _binned_threshold_check(threshold)


def _multilabel_binned_auprc_update_input_check(
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
