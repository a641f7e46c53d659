"""Recall, functional API (parity: functional/classification/recall.py:14-250).

The reference's macro/weighted path masks only ``num_tp`` (recall.py:190-195), which raises a
shape error whenever some class has neither labels nor predictions; here both operands are
masked (identical results whenever the reference succeeds).
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
def binary_recall(input: torch.Tensor, target: torch.Tensor, *, threshold: float = 0.5) -> torch.Tensor:
    """Recall of thresholded ``input`` vs ``target``.  Class: ``BinaryRecall``."""
    if _cpu_prf_ok(input, target):
        _binary_recall_update_input_check(input, target)
        out, warn = native().cpu_binary_prf(input, target, float(threshold), 1)
        if warn:
            logging.warning("No positive instances have been seen in target. Recall is converted from NaN to 0s.")
        return out
    num_tp, num_true_labels = _binary_recall_update(input, target, threshold)
    return _binary_recall_compute(num_tp, num_true_labels)


def _binary_recall_update(
    input: torch.Tensor, target: torch.Tensor, threshold: float = 0.5
) -> Tuple[torch.Tensor, torch.Tensor]:
    _binary_recall_update_input_check(input, target)
    if native_binary(input, target) and not target.is_floating_point():
        buf = torch.zeros(2, device=input.device)
        binary_counts(input, target, threshold=threshold, tp=buf[0:1], tp2=buf[1:2], fn=buf[1:2],
                      strict=True)
        return buf[0], buf[1]
    pred = torch.where(input < threshold, 0, 1)
    return (pred & target).sum(), target.sum()


def _binary_recall_compute(num_tp: torch.Tensor, num_true_labels: torch.Tensor) -> torch.Tensor:
    recall = num_tp / num_true_labels
    if torch.isnan(recall):
        logging.warning(
            "No positive instances have been seen in target. Recall is converted from NaN to 0s."
        )
        return torch.nan_to_num(recall)
    return recall


def _binary_recall_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")


def multiclass_recall(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_classes: Optional[int] = None,
    average: Optional[str] = "micro",
) -> torch.Tensor:
    """Recall for ``[N]`` labels or ``[N, C]`` scores; ``average`` in micro | macro |
    weighted | None.  Class version: ``MulticlassRecall``."""
    _recall_param_check(num_classes, average)
    if average in ("macro", "weighted"):
        _recall_update_input_check(input, target, num_classes)
        fast = cpu_class_metric(3, average, input, target, num_classes)
        if fast is not None:  # small CPU batch: one host call, no inference-mode context
            return _recall_fast(fast)
    return _multiclass_recall(input, target, num_classes, average)


@torch.inference_mode()
def _multiclass_recall(input, target, num_classes, average) -> torch.Tensor:
    num_tp, num_labels, num_predictions = _recall_update(input, target, num_classes, average)
    return _recall_compute(num_tp, num_labels, num_predictions, average)


def _recall_update(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int],
    average: Optional[str],
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _recall_update_input_check(input, target, num_classes)
    if native_cls(input, target):
        if average == "micro":
            buf = torch.zeros(2, device=input.device)
            cls_counts(input, target, micro_correct=buf[0:1], micro_total=buf[1:2])
            return buf[0], buf[1], buf[1]
        buf = torch.zeros(3, num_classes, device=input.device)
        cls_counts(input, target, num_classes=num_classes, cls_correct=buf[0], cls_label=buf[1],
                   cls_pred=buf[2])
        return buf[0], buf[1], buf[2]
    if input.ndim == 2:
        input = torch.argmax(input, dim=1)
    if average == "micro":
        num_tp = (input == target).sum()
        num_labels = target.new_tensor(target.numel())
        return num_tp, num_labels, num_labels
    hit = input == target
    ones = torch.ones_like(target)
    num_labels = target.new_zeros(num_classes).scatter_add_(0, target, ones)
    num_predictions = target.new_zeros(num_classes).scatter_add_(0, input, ones)
    num_tp = target.new_zeros(num_classes).scatter_add_(0, target[hit], ones[hit])
    return num_tp, num_labels, num_predictions


def _recall_compute(
    num_tp: torch.Tensor,
    num_labels: torch.Tensor,
    num_predictions: torch.Tensor,
    average: Optional[str],
) -> torch.Tensor:
    fast = cpu_class_average(3, average, num_tp, num_labels, num_predictions)
    if fast is not None:  # small CPU states: one host call
        return _recall_fast(fast)
    if average in ("macro", "weighted"):
        mask = (num_labels != 0) | (num_predictions != 0)
        num_tp = num_tp[mask]
        labels = num_labels[mask]
    else:
        labels = num_labels
    recall = num_tp / labels
    isnan_class = torch.isnan(recall)
    if isnan_class.any():
        nan_classes = isnan_class.nonzero(as_tuple=True)[0]
        logging.warning(
            f"One or more NaNs identified, as no ground-truth instances of {nan_classes.tolist()} have been seen. These have been converted to zero."
        )
        recall = torch.nan_to_num(recall)
    if average == "micro":
        return recall
    if average == "macro":
        return recall.mean()
    if average == "weighted":
        return (recall * (num_labels[mask] / num_labels.sum())).sum()
    return recall


def _recall_fast(fast) -> torch.Tensor:
    """The result of a host-call average (ops.classification.cpu_class_*), with the warning."""
    if fast[2]:
        logging.warning(
            f"One or more NaNs identified, as no ground-truth instances of {fast[2]} have been seen. These have been converted to zero."
        )
    return fast[0]


def _recall_param_check(num_classes: Optional[int], average: Optional[str]) -> None:
    average_options = ("micro", "macro", "weighted", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed values of {average_options}, got {average}."
        )
    if average != "micro" and (num_classes is None or num_classes <= 0):
        raise ValueError(
            f"`num_classes` should be a positive number when average={average}, got num_classes={num_classes}."
        )


def _recall_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]
) -> None:
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"`target` should be a one-dimensional tensor, got shape {target.shape}.")
    if input.ndim != 1 and not (
        input.ndim == 2 and (num_classes is None or input.shape[1] == num_classes)
    ):
        raise ValueError(
            f"`input` should have shape (num_samples,) or (num_samples, num_classes), got {input.shape}."
        )
