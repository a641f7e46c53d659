"""Recall at fixed precision, functional API (parity: recall_at_fixed_precision.py:24-156).

The reference builds every PR curve (per label in a Python loop) and then masks it twice per
label.  Here the answer is computed without materialising curves and without a host
synchronisation:

* ROCm: K3c's RAFP chain (csrc/kernels/curves.hip) - payload sort, count + scan, per-group
  recall / threshold with an atomic "last group meeting the precision", a device search for
  the first group reaching that recall, and a per-row finalize; all labels in one batch.
* elsewhere: ``_curve.recall_at_precision_rows``, the same selection vectorised over rows.

Semantics (reference :131-141): over the curve points (ascending thresholds plus the appended
precision 1 / recall 0 point, whose threshold counts as -1), the maximum recall among points
with precision >= ``min_precision``, and the absolute value of the highest threshold among the
points whose recall equals it.
"""

from typing import List, Tuple

import torch

from torcheval_amd.metrics.functional.classification._curve import recall_at_precision_rows
from torcheval_amd.metrics.functional.classification.precision_recall_curve import (
    _binary_precision_recall_curve_update_input_check,
    _multilabel_precision_recall_curve_update_input_check,
)
from torcheval_amd.ops import use_native

__all__ = ["binary_recall_at_fixed_precision", "multilabel_recall_at_fixed_precision"]


def _check_min_precision(min_precision: float) -> None:
    if not isinstance(min_precision, float) or not 0 <= min_precision <= 1:
        raise ValueError(
            f"Expected min_precision to be a float in the [0, 1] range but got {min_precision}."
        )


@torch.inference_mode()
def binary_recall_at_fixed_precision(
    input: torch.Tensor, target: torch.Tensor, *, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Highest recall whose precision is at least ``min_precision``, and its threshold, for
    ``[n]`` scores vs ``[n]`` {0, 1} targets.  Class version: ``BinaryRecallAtFixedPrecision``."""
    _binary_recall_at_fixed_precision_update_input_check(input, target, min_precision)
    return _binary_recall_at_fixed_precision_compute(input, target, min_precision)


def _binary_recall_at_fixed_precision_update_input_check(
    input: torch.Tensor, target: torch.Tensor, min_precision: float
) -> None:
    _binary_precision_recall_curve_update_input_check(input, target)
    _check_min_precision(min_precision)


def _rows_rafp(x: torch.Tensor, pos: torch.Tensor, min_precision: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """[rows, n] scores / boolean positives -> ([rows] max recall, [rows] |best threshold|);
    the threshold dtype follows the reference's cat with a float32 -1 (float32 or float64)."""
    best_dtype = torch.promote_types(x.dtype, torch.float32)
    if x.dtype in (torch.float16, torch.bfloat16):
        x = x.float()
    rec, thr = recall_at_precision_rows(x, pos, min_precision)
    return rec, thr.to(best_dtype)


def _binary_recall_at_fixed_precision_compute(
    input: torch.Tensor, target: torch.Tensor, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    if use_native(input) and target.is_cuda and input.numel() > 0:
        from torcheval_amd.ops.curves import binary_rafp

        return binary_rafp(input, target, min_precision)
    rec, thr = _rows_rafp(input.reshape(1, -1), (target == 1).reshape(1, -1), min_precision)
    return rec[0], thr[0]


@torch.inference_mode()
def multilabel_recall_at_fixed_precision(
    input: torch.Tensor, target: torch.Tensor, *, num_labels: int, min_precision: float
) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
    """Per-label (max recall, threshold) lists for ``[n, num_labels]`` data.
    Class version: ``MultilabelRecallAtFixedPrecision``."""
    if num_labels is None and input.ndim == 2:
        num_labels = input.shape[1]
    _multilabel_recall_at_fixed_precision_update_input_check(input, target, num_labels, min_precision)
    return _multilabel_recall_at_fixed_precision_compute(input, target, num_labels, min_precision)


def _multilabel_recall_at_fixed_precision_update_input_check(
    input: torch.Tensor, target: torch.Tensor, num_labels: int, min_precision: float
) -> None:
    _multilabel_precision_recall_curve_update_input_check(input, target, num_labels)
    _check_min_precision(min_precision)


def _multilabel_recall_at_fixed_precision_compute(
    input: torch.Tensor, target: torch.Tensor, num_labels: int, min_precision: float
) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
    if use_native(input) and target.is_cuda and input.shape[0] > 0:
        from torcheval_amd.ops.curves import multilabel_rafp

        rec, thr = multilabel_rafp(input, target, min_precision)
    else:
        rec, thr = _rows_rafp(input.t(), target.t() == 1, min_precision)
    return list(rec.unbind(0)), list(thr.unbind(0))


def _recall_at_precision(
    precision: torch.Tensor, recall: torch.Tensor, thresholds: torch.Tensor, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Selection on one already-built curve (``precision`` / ``recall`` carry the appended
    point, ``thresholds`` does not): device ops only, no boolean-mask compaction."""
    qual = precision >= min_precision
    max_recall = torch.where(qual, recall, torch.full_like(recall, -1.0)).amax()
    thr = thresholds.to(torch.promote_types(thresholds.dtype, torch.float32))
    thr = torch.cat([thr, thr.new_full((1,), -1.0)])
    cand = torch.where(recall == max_recall, thr, torch.full_like(thr, float("-inf")))
    return max_recall, cand.amax().abs()
