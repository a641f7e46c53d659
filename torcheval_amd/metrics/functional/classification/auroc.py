"""AUROC, functional API (parity: functional/classification/auroc.py:25-271).

Exact tie-aware AUROC.  ROCm: device sort + the fused K3 scan (no host sync).  The
reference's ``use_fbgemm`` switch (an approximate, tie-ignoring CUDA kernel from fbgemm_gpu)
is accepted for API compatibility; the exact K3 kernel is always used.
Return dtypes follow the reference: ``binary_auroc`` float64, ``multiclass_auroc`` float32.
"""

from typing import Optional

import torch

from torcheval_amd.metrics.functional.tensor_utils import _require_samples

from torcheval_amd.metrics.functional.classification._curve import binary_areas, multiclass_areas


@torch.inference_mode()
def binary_auroc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_tasks: int = 1,
    weight: Optional[torch.Tensor] = None,
    use_fbgemm: Optional[bool] = False,
) -> torch.Tensor:
    """
    Area under the ROC curve.  ``input``/``target`` are ``[n]`` or ``[num_tasks, n]``;
    optional ``weight`` of the same shape.  Class version: ``BinaryAUROC``.
    """
    _binary_auroc_update_input_check(input, target, num_tasks, weight)
    _require_samples(input.shape[-1] if input.ndim else 1, "binary_auroc")
    return _binary_auroc_compute(input, target, weight, use_fbgemm)


@torch.inference_mode()
def multiclass_auroc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    num_classes: int,
    average: Optional[str] = "macro",
) -> torch.Tensor:
    """One-vs-rest AUROC of ``[n, C]`` scores; ``average`` in macro | None.
    Class version: ``MulticlassAUROC``."""
    _multiclass_auroc_param_check(num_classes, average)
    _multiclass_auroc_update_input_check(input, target, num_classes)
    _require_samples(input.shape[0], "multiclass_auroc")
    return _multiclass_auroc_compute(input, target, num_classes, average)


def _binary_auroc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    weight: Optional[torch.Tensor] = None,
    use_fbgemm: Optional[bool] = False,
) -> torch.Tensor:
    roc, _ = binary_areas(input, target, weight, roc=True, pr=False)
    return roc[0] if input.dim() == 1 else roc


def _binary_auroc_update_input_check(
    input: torch.Tensor,
    target: torch.Tensor,
    num_tasks: int,
    weight: Optional[torch.Tensor] = None,
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            "The `input` and `target` should have the same shape, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if weight is not None and weight.shape != target.shape:
        raise ValueError(
            "The `weight` and `target` should have the same shape, "
            f"got shapes {weight.shape} and {target.shape}."
        )
    if num_tasks == 1:
        if len(input.shape) > 1:
            raise ValueError(
                f"`num_tasks = 1`, `input` is expected to be one-dimensional tensor, but got shape ({input.shape})."
            )
    elif len(input.shape) == 1 or input.shape[0] != num_tasks:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input`'s shape is expected to be ({num_tasks}, num_samples), but got shape ({input.shape})."
        )


def _multiclass_auroc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: int,
    average: Optional[str] = "macro",
) -> torch.Tensor:
    roc, _ = multiclass_areas(input, target, num_classes, roc=True, pr=False)
    roc = roc.to(torch.float32)
    if isinstance(average, str) and average == "macro":
        return roc.mean()
    return roc


def _multiclass_auroc_param_check(num_classes: int, average: Optional[str]) -> None:
    average_options = ("macro", "none", None)
    if average not in average_options:
        raise ValueError(
            f"`average` was not in the allowed value of {average_options}, got {average}."
        )
    if num_classes < 2:
        raise ValueError("`num_classes` has to be at least 2.")


def _multiclass_auroc_update_input_check(
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
