"""Accuracy family, functional API.

Parity: torcheval/metrics/functional/classification/accuracy.py (binary :13, multiclass :50,
multilabel :109, topk_multilabel :180; helpers :250-501, including the exact error strings).

ROCm tensors run the fused K1 kernel (csrc/kernels/classification.hip): one pass over the
[N, C] scores produces the correct/total counts (micro) or the per-class histograms
(macro / None) with no intermediate tensors.  CPU tensors run the ATen chain, which is
also the oracle in tests.  ``topk_multilabel_accuracy`` honours ``k`` (the reference
hard-codes ``topk(k=2)``, accuracy.py:407; identical for the default k=2).
"""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import compiling, native, native_loaded, use_native
from torcheval_amd.ops.classification import (
    binary_counts,
    cls_counts,
    cls_counts_supported,
    cpu_class_average,
    cpu_class_metric,
    multilabel_counts,
    native_cls,
    native_multilabel,
)


@torch.inference_mode()
def binary_accuracy(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: float = 0.5,
) -> torch.Tensor:
    """
    Frequency of thresholded ``input`` matching ``target``
    (``torch.where(input < threshold, 0, 1)`` is applied to ``input``).
    Class version: ``torcheval_amd.metrics.BinaryAccuracy``.
    """
    if _cpu_binary_ok(input, target):
        _binary_accuracy_update_input_check(input, target)
        return native().cpu_binary_accuracy(input, target, float(threshold))
    num_correct, num_total = _binary_accuracy_update(input, target, threshold)
    return _accuracy_compute(num_correct, num_total, "micro")


_CPU_TARGETS = (torch.bool, torch.uint8, torch.int32, torch.int64, torch.float32, torch.float64)


def _cpu_binary_ok(input: torch.Tensor, target: torch.Tensor) -> bool:
    """Small 1-D CPU batches go to the host twin (one C++ pass instead of ~5 ATen dispatches)."""
    return (
        input.device.type == "cpu"
        and target.device.type == "cpu"
        and input.dim() == 1
        and input.dtype in (torch.float32, torch.float64)
        and target.dtype in _CPU_TARGETS
        and input.numel() <= _CPU_FAST_MAX
        and not input.requires_grad
        and not compiling()
        and native_loaded()
    )


def multiclass_accuracy(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    average: Optional[str] = "micro",
    num_classes: Optional[int] = None,
    k: int = 1,
) -> torch.Tensor:
    """
    Frequency of ``input`` (labels ``[N]`` or scores ``[N, C]``, argmax'd) matching ``target``.

    ``average``: ``"micro"`` (global), ``"macro"`` (mean over classes that have samples) or
    ``None``/``"none"`` (per class, NaN for classes without samples).  ``k > 1`` counts a
    sample correct when its target is within the top-k scores.
    Class version: ``torcheval_amd.metrics.MulticlassAccuracy``.
    """
    if (
        average == "micro"
        and type(k) == int
        and k >= 1
        and not input.is_cuda
        and input.numel() <= _CPU_FAST_MAX
        and _cpu_fast_ok(input, target, k, num_classes)
    ):
        # small CPU batches: one fused C++ call instead of six ATen dispatches
        return native().cpu_micro_accuracy(input, target, k)
    if average == "macro" and type(k) == int and k >= 1:
        _accuracy_param_check(average, num_classes, k)
        _accuracy_update_input_check(input, target, num_classes, k)
        fast = cpu_class_metric(0, average, input, target, num_classes, k)
        if fast is not None:  # small CPU batch: one host call, no inference-mode context
            return fast[0]
    return _multiclass_accuracy_impl(input, target, average=average, num_classes=num_classes, k=k)


_CPU_FAST_MAX = 1 << 16


def _cpu_fast_ok(input: torch.Tensor, target: torch.Tensor, k: int, num_classes: Optional[int]) -> bool:
    if compiling() or not native_loaded() or target.dim() != 1 or target.dtype != torch.int64 or target.numel() == 0:
        return False
    if input.dim() == 2:
        ok = (
            input.dtype in (torch.float32, torch.float64)
            and input.shape[0] == target.shape[0]
            and input.stride(1) == 1
            and input.shape[1] > 0
            and (num_classes is None or input.shape[1] == num_classes)
        )
        return ok and (k == 1 or k <= input.shape[1]) and not input.requires_grad
    return input.dim() == 1 and k == 1 and input.dtype == torch.int64 and input.shape == target.shape


@torch.inference_mode()
def _multiclass_accuracy_impl(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    average: Optional[str],
    num_classes: Optional[int],
    k: int,
) -> torch.Tensor:
    _accuracy_param_check(average, num_classes, k)
    num_correct, num_total = _multiclass_accuracy_update(input, target, average, num_classes, k)
    return _accuracy_compute(num_correct, num_total, average)


@torch.inference_mode()
def multilabel_accuracy(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: float = 0.5,
    criteria: str = "exact_match",
) -> torch.Tensor:
    """
    Multilabel accuracy with ``criteria`` in ``exact_match`` | ``hamming`` | ``overlap`` |
    ``contain`` | ``belong``.  Class version: ``torcheval_amd.metrics.MultilabelAccuracy``.
    """
    _multilabel_accuracy_param_check(criteria)
    num_correct, num_total = _multilabel_accuracy_update(input, target, threshold, criteria)
    return _accuracy_compute(num_correct, num_total, "micro")


@torch.inference_mode()
def topk_multilabel_accuracy(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    criteria: str = "exact_match",
    k: int = 2,
) -> torch.Tensor:
    """
    Multilabel accuracy of the top-``k`` scored labels against ``target``.
    Class version: ``torcheval_amd.metrics.TopKMultilabelAccuracy``.
    """
    _topk_multilabel_accuracy_param_check(criteria, k)
    num_correct, num_total = _topk_multilabel_accuracy_update(input, target, criteria, k)
    return _accuracy_compute(num_correct, num_total, "micro")


# ----------------------------------------------------------------------------- updates
def _multiclass_accuracy_update(
    input: torch.Tensor,
    target: torch.Tensor,
    average: Optional[str],
    num_classes: Optional[int],
    k: int,
) -> Tuple[torch.Tensor, torch.Tensor]:
    _accuracy_update_input_check(input, target, num_classes, k)
    if use_native(input) and cls_counts_supported(input, target):
        dev = input.device
        if average == "micro":
            buf = torch.zeros(2, dtype=torch.float32, device=dev)
            cls_counts(input, target, k=k, num_classes=input.shape[1] if input.ndim == 2 else 0,
                       micro_correct=buf[0:1], micro_total=buf[1:2])
            return buf[0], buf[1]
        buf = torch.zeros(2, num_classes, dtype=torch.float32, device=dev)
        cls_counts(input, target, k=k, num_classes=num_classes,
                   cls_correct=buf[0], cls_label=buf[1])
        return buf[0], buf[1]
    if average != "micro" and not input.is_cuda and native_cls(input, target, num_classes=num_classes):
        # small CPU batches: the host twin of K1 fills both class histograms in one C++ call
        # (the ATen chain is argmax, eq, two scatter_adds and their zero / ones tensors)
        buf = torch.zeros(2, num_classes, dtype=torch.float32)
        cls_counts(input, target, k=k, num_classes=num_classes, cls_correct=buf[0], cls_label=buf[1])
        return buf[0], buf[1]
    return _multiclass_accuracy_update_aten(input, target, average, num_classes, k)


def _multiclass_accuracy_update_aten(
    input: torch.Tensor,
    target: torch.Tensor,
    average: Optional[str],
    num_classes: Optional[int],
    k: int,
) -> Tuple[torch.Tensor, torch.Tensor]:
    if k == 1:
        pred = input.argmax(dim=1) if input.ndim == 2 else input
        mask = (pred == target).long()
    else:
        target_score = input.gather(-1, target.unsqueeze(-1))
        mask = ((input > target_score).sum(dim=-1) < k).float()
    if average == "micro":
        return mask.sum(), torch.tensor(target.shape[0])
    num_correct = mask.new_zeros(num_classes).scatter_add_(0, target, mask)
    num_total = target.new_zeros(num_classes).scatter_add_(0, target, torch.ones_like(target))
    return num_correct, num_total


def _accuracy_compute(
    num_correct: torch.Tensor,
    num_total: torch.Tensor,
    average: Optional[str],
) -> torch.Tensor:
    if isinstance(average, str) and average == "macro":
        fast = cpu_class_average(0, average, num_correct, num_total)
        if fast is not None:  # small CPU states: one host call
            return fast[0]
        mask = num_total != 0
        return (num_correct[mask] / num_total[mask]).mean()
    return num_correct / num_total


def _accuracy_param_check(average: Optional[str], num_classes: Optional[int], k: int) -> None:
    average_options = ("micro", "macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if average != "micro" and (num_classes is None or num_classes <= 0):
        raise ValueError(
            f"num_classes should be a positive number when average={average}."
            f" Got num_classes={num_classes}."
        )
    if type(k) != int:
        raise TypeError(f"Expected `k` to be an integer, but {type(k)} was provided.")
    if k < 1:
        raise ValueError(
            f"Expected `k` to be an integer greater than 0, but {k} was provided."
        )


def _accuracy_update_input_check(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int],
    k: int,
) -> None:
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(
            f"target should be a one-dimensional tensor, got shape {target.shape}."
        )
    if k > 1 and input.ndim != 2:
        raise ValueError(
            "input should have shape (num_sample, num_classes) for k > 1, "
            f"got shape {input.shape}."
        )
    if not input.ndim == 1 and not (
        input.ndim == 2 and (num_classes is None or input.shape[1] == num_classes)
    ):
        raise ValueError(
            "input should have shape of (num_sample,) or (num_sample, num_classes), "
            f"got {input.shape}."
        )


def _binary_accuracy_update(
    input: torch.Tensor,
    target: torch.Tensor,
    threshold: float = 0.5,
) -> Tuple[torch.Tensor, torch.Tensor]:
    _binary_accuracy_update_input_check(input, target)
    if use_native(input) and target.is_cuda:
        buf = torch.zeros(2, dtype=torch.float32, device=input.device)
        binary_counts(input, target, threshold=threshold, tp=buf[0:1], tn=buf[0:1], total=buf[1:2])
        return buf[0], buf[1]
    pred = torch.where(input < threshold, 0, 1)
    num_correct = (pred == target).sum()
    num_total = torch.tensor(target.shape[0], dtype=torch.int64, device=target.device)
    return num_correct, num_total


def _binary_accuracy_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if target.ndim != 1:
        raise ValueError(
            f"target should be a one-dimensional tensor, got shape {target.shape}."
        )


def _multilabel_accuracy_update(
    input: torch.Tensor,
    target: torch.Tensor,
    threshold: float = 0.5,
    criteria: str = "exact_match",
) -> Tuple[torch.Tensor, torch.Tensor]:
    _multilabel_accuracy_update_input_check(input, target)
    if native_multilabel(input, target):
        return _multilabel_native(input, target, threshold, 0, criteria)
    input_label = torch.where(input < threshold, 0, 1)
    return _multilabel_update(input_label, target, criteria)


def _multilabel_native(
    input: torch.Tensor, target: torch.Tensor, threshold: float, k: int, criteria: str
) -> Tuple[torch.Tensor, torch.Tensor]:
    # K2: one pass, counts straight into a device scalar (no [N, L] label matrix)
    out = torch.zeros(2, dtype=torch.float32, device=input.device)
    multilabel_counts(
        input, target, threshold=threshold, k=k, criteria=criteria, num_correct=out[0], num_total=out[1]
    )
    return out[0], out[1]


def _topk_multilabel_accuracy_update(
    input: torch.Tensor,
    target: torch.Tensor,
    criteria: str = "exact_match",
    k: int = 2,
) -> Tuple[torch.Tensor, torch.Tensor]:
    _topk_multilabel_accuracy_update_input_check(input, target, k)
    if native_multilabel(input, target, k):
        return _multilabel_native(input, target, 0.5, k, criteria)
    topk_idx = input.topk(k=k, dim=-1).indices
    input_label = torch.zeros(input.size(), device=input.device).scatter_(-1, topk_idx, 1.0)
    return _multilabel_update(input_label, target, criteria)


def _multilabel_update(
    input: torch.Tensor,
    target: torch.Tensor,
    criteria: str = "exact_match",
) -> Tuple[torch.Tensor, torch.Tensor]:
    n = target.shape[0]
    if criteria == "hamming":
        return (input == target).sum(), torch.tensor(target.numel(), device=target.device)
    if criteria == "exact_match":
        num_correct = (input == target).all(dim=1).sum()
    elif criteria == "overlap":
        both_pos = torch.logical_and(input == target, input == 1).any(dim=1)
        both_empty = torch.logical_and(input == 0, target == 0).all(dim=1)
        num_correct = both_pos.sum() + both_empty.sum()
    elif criteria == "contain":
        num_correct = ((input - target) >= 0).all(dim=1).sum()
    else:  # belong
        num_correct = ((input - target) <= 0).all(dim=1).sum()
    return num_correct, torch.tensor(n, device=target.device)


def _multilabel_accuracy_param_check(criteria: str) -> None:
    criteria_options = ("exact_match", "hamming", "overlap", "contain", "belong")
    if criteria not in criteria_options:
        raise ValueError(
            f"`criteria` was not in the allowed value of {criteria_options}, got {criteria}."
        )


def _topk_multilabel_accuracy_param_check(criteria: str, k: int) -> None:
    _multilabel_accuracy_param_check(criteria)
    if type(k) != int:
        raise TypeError(f"Expected `k` to be an integer, but {type(k)} was provided.")
    if k == 1:
        raise ValueError(
            f"Expected `k` to be an integer greater than 1, but {k} was provided. In such case, please use multilabel_accuracy metric."
        )
    if k < 1:
        raise ValueError(
            f"Expected `k` to be an integer greater than 1, but {k} was provided."
        )


def _multilabel_accuracy_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )


def _topk_multilabel_accuracy_update_input_check(
    input: torch.Tensor, target: torch.Tensor, k: int
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same dimensions, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if input.ndim != 2:
        raise ValueError(
            "input should have shape (num_sample, num_classes) for k > 1, "
            f"got shape {input.shape}."
        )
