"""Binned AUROC, functional API (parity: functional/classification/binned_auroc.py:17-256).

The reference materialises a [T, tasks, N] boolean prediction tensor (binned_auroc.py:
111-138); here the per-threshold TP/FP counts come from the K4 histogram kernel and the
trapezoid runs over the T+1 curve points.
"""

from typing import List, Optional, Tuple, Union

import torch

from torcheval_amd.metrics.functional.tensor_utils import _threshold_check, _create_threshold_tensor
from torcheval_amd.ops.binned import binned_counts, binned_finalize, binned_finalize_supported

DEFAULT_NUM_THRESHOLD = 200


@torch.inference_mode()
def binary_binned_auroc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_tasks: int = 1,
    threshold: Union[int, List[float], torch.Tensor] = DEFAULT_NUM_THRESHOLD,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """(AUROC, thresholds) with scores binned at ``threshold``.  Class: ``BinaryBinnedAUROC``."""
    threshold = _create_threshold_tensor(threshold, target.device)
    _binary_binned_auroc_param_check(num_tasks, threshold)
    _binary_binned_auroc_update_input_check(input, target, num_tasks, threshold)
    return _binary_binned_auroc_compute(input, target, threshold)


def _binned_trapz(tp: torch.Tensor, fp: torch.Tensor) -> torch.Tensor:
    """tp/fp: [T, R] counts at ascending thresholds -> float64 [R] AUROC over the binned curve."""
    if binned_finalize_supported(tp, fp):
        return binned_finalize(tp, fp, auroc=True)[0]
    tp = tp.to(torch.float64)
    fp = fp.to(torch.float64)
    zero = tp.new_zeros(1, tp.shape[1])
    tp_next = torch.cat([tp[1:], zero])
    fp_next = torch.cat([fp[1:], zero])
    area = ((fp - fp_next) * (tp + tp_next)).sum(0) / 2
    factor = tp[0] * fp[0]
    return torch.where(factor == 0, torch.full_like(area, 0.5), area / torch.where(factor == 0, torch.ones_like(factor), factor))


def _binary_binned_auroc_compute(
    input: torch.Tensor, target: torch.Tensor, threshold: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor]:
    x = input if input.ndim == 2 else input.unsqueeze(0)
    t = target if target.ndim == 2 else target.unsqueeze(0)
    tp, fp, _ = binned_counts(x.t(), t.t(), threshold, 0)
    auroc = _binned_trapz(tp, fp)
    # the reference keeps the task dim even for 1-D input: shape [1] (binned_auroc.py:111-138)
    return auroc, threshold


def _binary_binned_auroc_param_check(num_tasks: int, threshold: torch.Tensor) -> None:
    if num_tasks < 1:
        raise ValueError("`num_tasks` has to be at least 1.")
    _threshold_check(threshold)


def _binary_binned_auroc_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_tasks: int, threshold: torch.Tensor
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same shape, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if len(input.shape) > 2:
        raise ValueError(
            f"`input` is expected to be two dimensions or less, but got {len(input.shape)}D tensor."
        )
    if num_tasks == 1:
        if len(input.shape) > 1:
            raise ValueError(
                f"`num_tasks = 1`, `input` is expected to be one-dimensional tensor, but got shape {input.shape}."
            )
    elif len(input.shape) == 1 or input.shape[0] != num_tasks:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input`'s shape is expected to be ({num_tasks}, num_samples), but got shape ({input.shape})."
        )


@torch.inference_mode()
def multiclass_binned_auroc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_classes: int,
    threshold: Union[int, List[float], torch.Tensor] = DEFAULT_NUM_THRESHOLD,
    average: Optional[str] = "macro",
) -> Tuple[torch.Tensor, torch.Tensor]:
    """One-vs-rest binned AUROC.  Class: ``MulticlassBinnedAUROC``."""
    threshold = _create_threshold_tensor(threshold, target.device)
    _multiclass_binned_auroc_param_check(num_classes, threshold, average)
    _multiclass_binned_auroc_update_input_check(input, target, num_classes)
    return _multiclass_binned_auroc_compute(input, target, num_classes, threshold, average)


def _multiclass_binned_auroc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: int,
    threshold: torch.Tensor,
    average: Optional[str] = "macro",
) -> Tuple[torch.Tensor, torch.Tensor]:
    tp, fp, _ = binned_counts(input, target, threshold, 1)
    auroc = _binned_trapz(tp, fp).to(torch.float32)
    if isinstance(average, str) and average == "macro":
        return auroc.mean(), threshold
    return auroc, threshold


def _multiclass_binned_auroc_param_check(
    num_classes: int, threshold: torch.Tensor, average: Optional[str]
) -> None:
    average_options = ("macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if num_classes < 2:
        raise ValueError("`num_classes` has to be at least 2.")
    _threshold_check(threshold)


def _multiclass_binned_auroc_update_input_check(
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
