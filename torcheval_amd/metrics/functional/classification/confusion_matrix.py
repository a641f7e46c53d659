"""Confusion matrix, functional API (parity: functional/classification/confusion_matrix.py).

ROCm: K1 scatters (target, argmax) pairs straight into the [C, C] float matrix — the
reference builds ``vstack`` + ``sparse_coo_tensor`` + ``to_dense`` (confusion_matrix.py:
219-234) and host-syncs on ``torch.max(input/target)`` for validation every update
(:271-278).  On the GPU path out-of-range labels are flagged on device and raised without a
per-update sync (class metrics raise at ``compute()``).
"""

from typing import Optional

import torch
import torch.nn.functional as F

from torcheval_amd.ops.classification import binary_counts, cls_counts, cpu_confusion, native_binary, native_cls
from torcheval_amd.ops.hostread import read_int


@torch.inference_mode()
def binary_confusion_matrix(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: float = 0.5,
    normalize: Optional[str] = None,
) -> torch.Tensor:
    """2x2 confusion matrix (rows: target, cols: prediction) of thresholded ``input``.
    ``normalize`` in None | "none" | "true" | "pred" | "all".  Class: ``BinaryConfusionMatrix``."""
    _confusion_matrix_param_check(2, normalize)
    if normalize in (None, "none"):
        _binary_confusion_matrix_update_input_check(input, target)
        cm = cpu_confusion(input, target, 2, threshold, binary=True)
        if cm is not None:  # small CPU batch: one host call
            return cm
    matrix = _binary_confusion_matrix_update(input, target, threshold)
    return _functional_result(matrix, normalize)


@torch.inference_mode()
def multiclass_confusion_matrix(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: int,
    *,
    normalize: Optional[str] = None,
) -> torch.Tensor:
    """[C, C] confusion matrix (rows: target, cols: prediction).
    Class version: ``MulticlassConfusionMatrix``."""
    _confusion_matrix_param_check(num_classes, normalize)
    if normalize in (None, "none"):
        _confusion_matrix_shape_check(input, target, num_classes)
        cm = cpu_confusion(input, target, num_classes)
        if cm is not None:  # small CPU batch, labels in range: one host call
            return cm
    cm = _confusion_matrix_update(input, target, num_classes)
    return _functional_result(cm, normalize)


def _functional_result(cm: torch.Tensor, normalize: Optional[str]) -> torch.Tensor:
    """Un-normalised functional results are int64 counts as in the reference (its bincount /
    sparse path); the K1 kernel accumulates exact integer-valued f32 counts."""
    if normalize in (None, "none") and cm.is_floating_point():
        return cm.long()
    return _confusion_matrix_compute(cm, normalize=normalize)


def _binary_confusion_matrix_compute(cm: torch.Tensor, normalize: Optional[str]) -> torch.Tensor:
    # kept for API parity (reference :152-162, unused there as well)
    if normalize == "pred":
        return F.normalize(cm.to(torch.float), p=1, dim=1)
    if normalize == "true":
        return F.normalize(cm.to(torch.float), p=1, dim=0)
    if normalize == "all":
        return cm.to(torch.float) / torch.sum(cm)
    return cm


def _binary_confusion_matrix_update(
    input: torch.Tensor, target: torch.Tensor, threshold: float = 0.5
) -> torch.Tensor:
    _binary_confusion_matrix_update_input_check(input, target)
    if native_binary(input, target) and not target.is_floating_point():
        cm = torch.zeros(2, 2, device=input.device)
        flat = cm.view(-1)
        binary_counts(input, target, threshold=threshold, tn=flat[0:1], fp=flat[1:2],
                      fn=flat[2:3], tp=flat[3:4], strict=True)
        return cm
    pred = torch.where(input < threshold, 0, 1)
    return _dense_update(pred, target, 2)


def _binary_confusion_matrix_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.ndim != 1:
        raise ValueError(
            f"input should be a one-dimensional tensor for binary confusion matrix, got shape {input.shape}."
        )
    if target.ndim != 1:
        raise ValueError(
            f"target should be a one-dimensional tensor for binary confusion matrix, got shape {target.shape}."
        )
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )


def _confusion_matrix_compute(confusion_matrix: torch.Tensor, normalize: Optional[str]) -> torch.Tensor:
    if normalize == "pred":
        return F.normalize(confusion_matrix.to(torch.float), p=1, dim=0)
    if normalize == "true":
        return F.normalize(confusion_matrix.to(torch.float), p=1, dim=1)
    if normalize == "all":
        return confusion_matrix.to(torch.float) / torch.sum(confusion_matrix)
    return confusion_matrix


def _confusion_matrix_update(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: int,
    err: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """Dense [C, C] counts.  GPU path validates on device: pass ``err`` (int32[1]) to collect
    the flag; without it the flag is checked here (one sync, like the reference's check)."""
    # an empty batch takes the checking path: the reference's torch.max check raises on it
    if native_cls(input, target) and input.shape[0] > 0:
        _confusion_matrix_shape_check(input, target, num_classes)
        cm = torch.zeros(num_classes, num_classes, device=input.device)
        own_err = err is None
        if own_err:
            err = torch.zeros(1, dtype=torch.int32, device=input.device)
        cls_counts(input, target, num_classes=num_classes, confusion=cm.view(-1), err=err)
        if own_err:
            _raise_confusion_err(err, input, target, num_classes)
        return cm
    _confusion_matrix_update_input_check(input, target, num_classes)
    return _dense_update(input, target, num_classes)


def _raise_confusion_err(err: torch.Tensor, input, target, num_classes: int) -> None:
    code = read_int(err)
    if code & 2:
        raise ValueError(
            "Got `input` prediction class which is too large for the number of classes, "
            f"num_classes: {num_classes} must be strictly greater than max class predicted: {torch.max(input)}."
        )
    if code & 1:
        raise ValueError(
            "Got `target` class which is larger than the number of classes, "
            f"num_classes: {num_classes} must be strictly greater than max target: {torch.max(target)}."
        )


def _dense_update(input: torch.Tensor, target: torch.Tensor, num_classes: int) -> torch.Tensor:
    if input.ndim == 2:
        input = torch.argmax(input, dim=1)
    flat = target.long() * num_classes + input.long()
    return torch.bincount(flat, minlength=num_classes * num_classes).view(num_classes, num_classes)


def _confusion_matrix_param_check(num_classes: int, normalize: Optional[str]) -> None:
    if num_classes < 2:
        raise ValueError("Must be at least two classes for confusion matrix")
    if normalize is not None and normalize not in ["all", "pred", "true", "none"]:
        raise ValueError("normalize must be one of 'all', 'pred', 'true', or 'none'.")


def _confusion_matrix_shape_check(input: torch.Tensor, target: torch.Tensor, num_classes: int) -> None:
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
    if not input.ndim == 1 and not (input.ndim == 2 and input.shape[1] == num_classes):
        raise ValueError(
            f"input should have shape of (num_sample,) or (num_sample, num_classes), got {input.shape}."
        )


def _confusion_matrix_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]
) -> None:
    _confusion_matrix_shape_check(input, target, num_classes)
    if input.ndim == 1 and torch.max(input) >= num_classes:
        raise ValueError(
            "Got `input` prediction class which is too large for the number of classes, "
            f"num_classes: {num_classes} must be strictly greater than max class predicted: {torch.max(input)}."
        )
    if torch.max(target) >= num_classes:
        raise ValueError(
            "Got `target` class which is larger than the number of classes, "
            f"num_classes: {num_classes} must be strictly greater than max target: {torch.max(target)}."
        )
