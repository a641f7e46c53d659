"""Precision, functional API (parity: functional/classification/precision.py:17-250).

ROCm tensors: one K1 launch produces tp / fp / label counts (micro: correct & wrong rows;
per-class: correct at target, rows per target, wrong rows per predicted class).
"""

import logging
from typing import Optional, Tuple

import torch

from torcheval_amd.ops import native
from torcheval_amd.ops.classification import (
    _cpu_prf_ok,
    binary_counts,
    cls_counts,
    cpu_class_average,
    cpu_class_metric,
    native_binary,
    native_cls,
)


@torch.inference_mode()
def binary_precision(input: torch.Tensor, target: torch.Tensor, *, threshold: float = 0.5) -> torch.Tensor:
    """Precision of thresholded ``input`` (``input >= threshold`` is positive) vs ``target``.
    Class version: ``torcheval_amd.metrics.BinaryPrecision``."""
    if _cpu_prf_ok(input, target):
        _binary_precision_update_input_check(input, target)
        return native().cpu_binary_prf(input, target, float(threshold), 0)[0]
    num_tp, num_fp, num_label = _binary_precision_update(input, target, threshold)
    return _precision_compute(num_tp, num_fp, num_label, "micro")


def multiclass_precision(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_classes: Optional[int] = None,
    average: Optional[str] = "micro",
) -> torch.Tensor:
    """Precision for ``[N]`` labels or ``[N, C]`` scores; ``average`` in micro | macro |
    weighted | None.  Class version: ``torcheval_amd.metrics.MulticlassPrecision``."""
    _precision_param_check(num_classes, average)
    if average in ("macro", "weighted"):
        _precision_update_input_check(input, target, num_classes)
        fast = cpu_class_metric(2, average, input, target, num_classes)
        if fast is not None:  # small CPU batch: one host call, no inference-mode context
            return fast[0]
    return _multiclass_precision(input, target, num_classes, average)


@torch.inference_mode()
def _multiclass_precision(input, target, num_classes, average) -> torch.Tensor:
    num_tp, num_fp, num_label = _precision_update(input, target, num_classes, average)
    return _precision_compute(num_tp, num_fp, num_label, average)


def _precision_update(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int],
    average: Optional[str],
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _precision_update_input_check(input, target, num_classes)
    if native_cls(input, target):
        if average == "micro":
            buf = torch.zeros(2, device=input.device)
            cls_counts(input, target, micro_correct=buf[0:1], micro_incorrect=buf[1:2])
            return buf[0], buf[1], torch.tensor(0.0)
        buf = torch.zeros(3, num_classes, device=input.device)
        cls_counts(input, target, num_classes=num_classes, cls_correct=buf[0], cls_fp=buf[1],
                   cls_label=buf[2])
        return buf[0], buf[1], buf[2]
    if input.ndim == 2:
        input = torch.argmax(input, dim=1)
    if average == "micro":
        return (input == target).sum(), (input != target).sum(), torch.tensor(0.0)
    # hit / miss as 0/1 scatter weights (no boolean-mask indexing: static shapes, traceable by
    # torch.compile, same counts)
    hit = (input == target).to(target.dtype)
    num_label = target.new_zeros(num_classes).scatter_add_(0, target, torch.ones_like(target))
    num_tp = target.new_zeros(num_classes).scatter_add_(0, target, hit)
    num_fp = target.new_zeros(num_classes).scatter_add_(0, input, 1 - hit)
    return num_tp, num_fp, num_label


def _precision_compute(
    num_tp: torch.Tensor,
    num_fp: torch.Tensor,
    num_label: torch.Tensor,
    average: Optional[str],
) -> torch.Tensor:
    fast = cpu_class_average(2, average, num_tp, num_fp, num_label)
    if fast is not None:  # small CPU states: one host call
        return fast[0]
    if average in ("macro", "weighted"):
        mask = (num_label != 0) | (num_tp + num_fp != 0)
        num_tp, num_fp = num_tp[mask], num_fp[mask]
    precision = num_tp / (num_tp + num_fp)
    if average in (None, "None") and torch.isnan(precision).any():
        bad_class = torch.nonzero(torch.isnan(precision))
        logging.warning(
            f"{bad_class} classes have zero instances in both the predictions and the ground truth labels. Precision is still logged as zero."
        )
    precision = torch.nan_to_num(precision)
    if average == "micro":
        return precision
    if average == "macro":
        return precision.mean()
    if average == "weighted":
        return torch.inner(precision, num_label[mask] / num_label.sum())
    return precision


def _precision_param_check(num_classes: Optional[int], average: Optional[str]) -> None:
    average_options = ("micro", "macro", "weighted", "None", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if average != "micro" and (num_classes is None or num_classes <= 0):
        raise ValueError(
            f"num_classes should be a positive number when average={average}. Got num_classes={num_classes}."
        )


def _precision_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]
) -> None:
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
    if not input.ndim == 1 and not (
        input.ndim == 2 and (num_classes is None or input.shape[1] == num_classes)
    ):
        raise ValueError(
            f"input should have shape of (num_sample,) or (num_sample, num_classes), got {input.shape}."
        )


def _binary_precision_update(
    input: torch.Tensor, target: torch.Tensor, threshold: float = 0.5
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _binary_precision_update_input_check(input, target)
    if native_binary(input, target) and not target.is_floating_point():
        buf = torch.zeros(2, device=input.device)
        binary_counts(input, target, threshold=threshold, tp=buf[0:1], fp=buf[1:2])
        return buf[0], buf[1], torch.tensor(0.0)
    pred = torch.where(input < threshold, 0, 1)
    num_tp = (pred * target).sum(dim=-1)
    num_fp = pred.sum(dim=-1) - num_tp
    return num_tp, num_fp, torch.tensor(0.0)


def _binary_precision_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
