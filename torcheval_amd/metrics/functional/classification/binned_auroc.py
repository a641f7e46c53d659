"""Binned AUROC, functional API (parity: functional/classification/binned_auroc.py:17-256).

``multiclass_binned_auroc`` reproduces the reference's per-sample rows by default and offers
per-class one-vs-rest as ``one_vs_rest=True`` (docs/parity.md).

The reference materialises a [T, tasks, N] boolean prediction tensor (binned_auroc.py:
111-138); here the per-threshold TP/FP counts come from the K4 histogram kernel and the
trapezoid runs over the T+1 curve points.
"""

from typing import List, Optional, Tuple, Union

import torch

from torcheval_amd.metrics.functional.tensor_utils import _threshold_check, _create_threshold_tensor
from torcheval_amd.ops import native, use_native
from torcheval_amd.ops.binned import binned_counts, binned_finalize, binned_finalize_supported
from torcheval_amd.ops.hostread import read_int

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
    one_vs_rest: bool = False,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Binned AUROC for multiclass scores.  Class: ``MulticlassBinnedAUROC``.

    By default this returns exactly what the reference returns (binned_auroc.py:188-215): the
    one-hot product is summed over the CLASS dim, so each row of the curve is one SAMPLE (its
    true-class score as the single positive, its other classes as negatives), and ``average=None``
    gives one value per sample.  The reference's own example: ``tensor(0.4000)`` and the
    5-vector ``[0.5, 0.25, 0.25, 0.0, 1.0]`` for 5 samples x 3 classes.

    ``one_vs_rest=True`` opts into per-class one-vs-rest binned AUROC (one value per class;
    at thresholds that cover every score it equals the exact ``multiclass_auroc``), computed
    from the K4 histogram kernel.
    """
    threshold = _create_threshold_tensor(threshold, target.device)
    _multiclass_binned_auroc_param_check(num_classes, threshold, average)
    _multiclass_binned_auroc_update_input_check(input, target, num_classes)
    return _multiclass_binned_auroc_compute(input, target, num_classes, threshold, average, one_vs_rest)


def _native_per_sample(input: torch.Tensor, target: torch.Tensor, num_classes: int, threshold: torch.Tensor) -> bool:
    return (
        use_native(input)
        and input.dim() == 2
        and input.dtype == torch.float32
        and input.shape[1] == num_classes
        and input.shape[1] >= 1
        and input.stride(1) == 1
        and input.shape[0] > 0
        and threshold.dtype == torch.float32
        and threshold.numel() >= 1
        and target.is_cuda
        and target.dim() == 1
        and not target.dtype.is_floating_point
    )


def _per_sample_binned_auroc(input: torch.Tensor, target: torch.Tensor, num_classes: int,
                             threshold: torch.Tensor) -> torch.Tensor:
    """float32 [N]: the reference's per-sample rows, without its [T, N, C] boolean tensor.

    Each score's bin b = #{t : score >= thr_t} (one searchsorted); per sample, the count of
    classes at or above thr_t is the suffix sum of a [T + 1] histogram of its bins; the true
    class contributes tp_t = [t < b_true] and the rest fp_t.  The trapezoid runs over the
    descending-threshold curve with a leading 0, as ``rot90`` + ``pad`` build it there."""
    if _native_per_sample(input, target, num_classes, threshold):
        # K4b (csrc/kernels/binned_auroc.hip): one streaming pass, one binary search per
        # sample; the label range goes through a device flag read once (no min / max syncs)
        out = torch.empty(input.shape[0], dtype=torch.float32, device=input.device)
        err = torch.zeros(1, dtype=torch.int32, device=input.device)
        t = target if target.dtype in (torch.int64, torch.int32) else target.long()
        native().sample_binned_auroc(input, t, threshold.to(input.device).contiguous(), out, err)
        if read_int(err):
            raise RuntimeError("Class values must be smaller than num_classes.")  # F.one_hot's check
        return out
    if target.numel() and (int(target.min()) < 0 or int(target.max()) >= num_classes):
        raise RuntimeError("Class values must be smaller than num_classes.")  # F.one_hot's check
    n, T = input.shape[0], threshold.numel()
    dev = input.device
    dt = torch.promote_types(input.dtype, threshold.dtype)
    thr = threshold.to(device=dev, dtype=dt).contiguous()
    out = torch.empty(n, dtype=torch.float32, device=dev)
    ar = torch.arange(T, device=dev)
    step = max(1, (1 << 24) // max(T + 1, num_classes))  # bounds the [rows, T + 1] temporaries
    for s0 in range(0, n, step):
        x = input[s0 : s0 + step].to(dt)
        rows = x.shape[0]
        b = torch.searchsorted(thr, x.contiguous(), right=True)
        b = torch.where(torch.isnan(x), torch.zeros_like(b), b)  # NaN >= thr is false
        hist = torch.zeros(rows, T + 1, dtype=torch.int64, device=dev).scatter_add_(1, b, torch.ones_like(b))
        ge = hist.flip(1).cumsum(1).flip(1)[:, 1:]  # [rows, T]: classes with score >= thr_t
        b_true = b.gather(1, target[s0 : s0 + step].long().view(-1, 1))
        tp = (ar.view(1, -1) < b_true).to(torch.int64)
        fp = ge - tp
        zero = torch.zeros(rows, 1, dtype=torch.int64, device=dev)
        tpd = torch.cat([zero, tp.flip(1)], 1).to(torch.float64)
        fpd = torch.cat([zero, fp.flip(1)], 1).to(torch.float64)
        area = ((fpd[:, 1:] - fpd[:, :-1]) * (tpd[:, 1:] + tpd[:, :-1])).sum(1) / 2  # exact
        factor = (tp[:, 0] * fp[:, 0]).to(torch.float32)
        res = area.to(torch.float32) / torch.where(factor == 0, torch.ones_like(factor), factor)
        out[s0 : s0 + rows] = torch.where(factor == 0, torch.full_like(res, 0.5), res)
    return out


def _multiclass_binned_auroc_compute(
    input: torch.Tensor,
    target: torch.Tensor,
    num_classes: int,
    threshold: torch.Tensor,
    average: Optional[str] = "macro",
    one_vs_rest: bool = False,
) -> Tuple[torch.Tensor, torch.Tensor]:
    if one_vs_rest:
        tp, fp, _ = binned_counts(input, target, threshold, 1)
        auroc = _binned_trapz(tp, fp).to(torch.float32)
    else:
        auroc = _per_sample_binned_auroc(input, target, num_classes, threshold)
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
