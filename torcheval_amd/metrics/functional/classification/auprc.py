"""AUPRC (average precision), functional API (parity: functional/classification/auprc.py).

The reference builds a full PR curve per task / class in a Python loop, then a Riemann sum
and a CPU round trip through ``torch.tensor(list)`` (auprc.py:239-347).  Here every row is
integrated in one pass (K3 on ROCm, vectorised FP64 ATen on CPU).  Results are float32 like
the reference's.
"""

from typing import Optional

import torch

from torcheval_amd.metrics.functional.tensor_utils import _require_samples

from torcheval_amd.metrics.functional.classification._curve import binary_areas, multiclass_areas


@torch.inference_mode()
def binary_auprc(input: torch.Tensor, target: torch.Tensor, *, num_tasks: int = 1) -> torch.Tensor:
    """Area under the precision-recall curve of ``[n]`` / ``[num_tasks, n]`` data.
    Class version: ``BinaryAUPRC``."""
    _binary_auprc_update_input_check(input, target, num_tasks)
    _require_samples(input.shape[-1] if input.ndim else 1, "binary_auprc")
    return _binary_auprc_compute(input, target, num_tasks)


@torch.inference_mode()
def multiclass_auprc(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: Optional[int] = None,
    *,
    average: Optional[str] = "macro",
) -> torch.Tensor:
    """One-vs-rest AUPRC of ``[n, C]`` scores vs ``[n]`` labels; ``average`` in macro | None.
    Class version: ``MulticlassAUPRC``."""
    if num_classes is None:
        num_classes = input.shape[1]
    _multiclass_auprc_param_check(num_classes, average)
    _multiclass_auprc_update_input_check(input, target, num_classes)
    _require_samples(input.shape[0], "multiclass_auprc")
    return _multiclass_auprc_compute(input, target, average, num_classes)


@torch.inference_mode()
def multilabel_auprc(
    input: torch.Tensor,
    target: torch.Tensor,
    num_labels: Optional[int] = None,
    *,
    average: Optional[str] = "macro",
) -> torch.Tensor:
    """Per-label AUPRC of ``[n, L]`` scores vs ``[n, L]`` {0,1} targets.
    Class version: ``MultilabelAUPRC``."""
    if input.ndim != 2:
        raise ValueError(f"input should be a two-dimensional tensor, got shape {input.shape}.")
    if num_labels is None:
        num_labels = input.shape[1]
    _multilabel_auprc_param_check(num_labels, average)
    _multilabel_auprc_update_input_check(input, target, num_labels)
    return _multilabel_auprc_compute(input, target, num_labels, average)


def _binary_auprc_compute(input: torch.Tensor, target: torch.Tensor, num_tasks: int = 1) -> torch.Tensor:
    _, pr = binary_areas(input, target, None, roc=False, pr=True)
    pr = pr.to(torch.float32)
    if num_tasks == 1 and input.ndim == 1:
        return pr[0]
    return pr


def _binary_auprc_update_input_check(input: torch.Tensor, target: torch.Tensor, num_tasks: int) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same shape, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if num_tasks == 1:
        if input.ndim == 2 and input.shape[0] > 1 or input.ndim > 2:
            raise ValueError(
                f"`num_tasks = 1`, `input` and `target` are expected to be one-dimensional tensors or 1xN tensors, but got shape input: {input.shape}, target: {target.shape}."
            )
    elif input.shape[0] != num_tasks:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input` and `target` shape is expected to be ({num_tasks}, num_samples), but got shape input: {input.shape}, target: {target.shape}."
        )


def _multiclass_auprc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    average: Optional[str] = "macro",
    num_classes: Optional[int] = None,
) -> torch.Tensor:
    num_classes = input.shape[1] if num_classes is None else num_classes
    _, pr = multiclass_areas(input, target, num_classes, roc=False, pr=True)
    pr = pr.to(torch.float32)
    return pr.mean() if average == "macro" else pr


def _multiclass_auprc_param_check(num_classes: int, average: Optional[str]) -> None:
    average_options = ("macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if num_classes < 2:
        raise ValueError("`num_classes` has to be at least 2.")


def _multiclass_auprc_update_input_check(
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


def _multilabel_auprc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    num_labels: int,
    average: Optional[str] = "macro",
) -> torch.Tensor:
    _, pr = binary_areas(input.t(), target.t(), None, roc=False, pr=True)
    pr = pr.to(torch.float32)
    return pr.mean() if average == "macro" else pr


def _multilabel_auprc_param_check(num_labels: int, average: Optional[str]) -> None:
    average_options = ("macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if num_labels < 2:
        raise ValueError("`num_labels` has to be at least 2.")


def _multilabel_auprc_update_input_check(
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
