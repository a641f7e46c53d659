"""F1 score, functional API (parity: functional/classification/f1_score.py:16-273)."""

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
def binary_f1_score(input: torch.Tensor, target: torch.Tensor, *, threshold: float = 0.5) -> torch.Tensor:
    """F1 of thresholded ``input`` vs ``target``.  Class version: ``BinaryF1Score``."""
    if _cpu_prf_ok(input, target):
        _binary_f1_score_update_input_check(input, target)
        out, warn = native().cpu_binary_prf(input, target, float(threshold), 2)
        if warn:
            logging.warning(
                "Warning: Some classes do not exist in the target. F1 scores for these classes will be cast to zeros."
            )
        return out
    num_tp, num_label, num_prediction = _binary_f1_score_update(input, target, threshold)
    return _f1_score_compute(num_tp, num_label, num_prediction, "micro")


def multiclass_f1_score(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_classes: Optional[int] = None,
    average: Optional[str] = "micro",
) -> torch.Tensor:
    """F1 for ``[N]`` labels or ``[N, C]`` scores; ``average`` in micro | macro | weighted |
    None.  Class version: ``MulticlassF1Score``."""
    _f1_score_param_check(num_classes, average)
    if average in ("macro", "weighted"):
        _f1_score_update_input_check(input, target, num_classes)
        fast = cpu_class_metric(1, average, input, target, num_classes)
        if fast is not None:  # small CPU batch: one host call, no inference-mode context
            return _f1_fast(fast)
    return _multiclass_f1_score(input, target, num_classes, average)


@torch.inference_mode()
def _multiclass_f1_score(input, target, num_classes, average) -> torch.Tensor:
    num_tp, num_label, num_prediction = _f1_score_update(input, target, num_classes, average)
    return _f1_score_compute(num_tp, num_label, num_prediction, average)


def _binary_f1_score_update(
    input: torch.Tensor, target: torch.Tensor, threshold: float = 0.5
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _binary_f1_score_update_input_check(input, target)
    if native_binary(input, target) and not target.is_floating_point():
        buf = torch.zeros(3, device=input.device)
        # tp -> (tp, label), fn -> label, fp -> prediction, and tp also -> prediction
        binary_counts(input, target, threshold=threshold, tp=buf[0:1], tp2=buf[1:2],
                      fn=buf[1:2], fp=buf[2:3], strict=True)
        buf[2] += buf[0]
        return buf[0], buf[1], buf[2]
    pred = torch.where(input < threshold, 0, 1)
    return (pred * target).sum(), target.sum(), pred.sum()


def _binary_f1_score_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.ndim != 1:
        raise ValueError(
            f"input should be a one-dimensional tensor for binary f1 score, got shape {input.shape}."
        )
    if target.ndim != 1:
        raise ValueError(
            f"target should be a one-dimensional tensor for binary f1 score, got shape {target.shape}."
        )
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )


def _f1_score_update(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int],
    average: Optional[str],
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _f1_score_update_input_check(input, target, num_classes)
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
        num_label = torch.tensor(target.shape[0], device=target.device)
        return num_tp, num_label, num_label
    hit = input == target
    ones = torch.ones(target.shape[0], device=target.device)
    num_label = torch.zeros(num_classes, device=target.device).scatter_add_(0, target, ones)
    num_prediction = torch.zeros(num_classes, device=target.device).scatter_add_(0, input, ones)
    num_tp = torch.zeros(num_classes, device=target.device).scatter_add_(0, target[hit], ones[hit])
    return num_tp, num_label, num_prediction


def _f1_score_compute(
    num_tp: torch.Tensor,
    num_label: torch.Tensor,
    num_prediction: torch.Tensor,
    average: Optional[str],
) -> torch.Tensor:
    fast = cpu_class_average(1, average, num_tp, num_label, num_prediction)
    if fast is not None:  # small CPU states: one host call
        return _f1_fast(fast)
    num_label_is_zero = num_label == 0
    if num_label_is_zero.any():
        logging.warning(
            "Warning: Some classes do not exist in the target. F1 scores for these classes will be cast to zeros."
        )
    if average in ("macro", "weighted"):
        mask = ~num_label_is_zero | (num_prediction != 0)
        num_tp, num_label, num_prediction = num_tp[mask], num_label[mask], num_prediction[mask]
    precision = num_tp / num_prediction
    recall = num_tp / num_label
    f1 = torch.nan_to_num(2 * precision * recall / (precision + recall))
    if average == "micro":
        return f1
    if average == "macro":
        return f1.mean()
    if average == "weighted":
        return (f1 * (num_label / num_label.sum())).sum()
    return f1


def _f1_fast(fast) -> torch.Tensor:
    """The result of a host-call average (ops.classification.cpu_class_*), with the warning."""
    if fast[1]:
        logging.warning(
            "Warning: Some classes do not exist in the target. F1 scores for these classes will be cast to zeros."
        )
    return fast[0]


def _f1_score_param_check(num_classes: Optional[int], average: Optional[str]) -> None:
    average_options = ("micro", "macro", "weighted", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if average != "micro" and (num_classes is None or num_classes <= 0):
        raise ValueError(
            f"num_classes should be a positive number when average={average}, got num_classes={num_classes}."
        )


def _f1_score_update_input_check(
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
