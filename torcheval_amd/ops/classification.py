"""Python wrappers of the K1 classification-count kernels (csrc/kernels/classification.hip).

All wrappers accumulate INTO caller-provided float32 tensors (metric states or fresh zero
buffers), so a class-metric ``update()`` is exactly one kernel launch.
"""

from typing import Optional

import torch

import torcheval_amd.ops as _ops
from torcheval_amd.ops import MAX_BLOCKS, compiling, native, native_loaded, use_native

_SCORE_DTYPES = (torch.float32, torch.bfloat16, torch.float16)
_LABEL_DTYPES = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)
_BINARY_DTYPES = _LABEL_DTYPES + (torch.float32, torch.float16, torch.bfloat16, torch.float64)


def cls_counts_supported(input: torch.Tensor, target: torch.Tensor) -> bool:
    """Whether the fused kernel handles this (input, target) dtype/shape combination."""
    if target.dtype not in _LABEL_DTYPES or target.dim() != 1:
        return False
    if input.dim() == 2:
        return input.dtype in _SCORE_DTYPES
    if input.dim() == 1:
        return input.dtype in _LABEL_DTYPES
    return False


# CPU batches up to this many scores take the host twin of K1 (csrc/runtime/cpu_metrics.cpp):
# one C++ call instead of ~6-10 ATen dispatches, which dominate small updates
_CPU_MAX = 1 << 16


def _cpu_cls(input: torch.Tensor, target: torch.Tensor, num_classes: Optional[int]) -> bool:
    if compiling() or input.is_cuda or target.is_cuda or _ops.DISABLE_HIP or not native_loaded():
        return False
    if input.numel() > _CPU_MAX or target.dim() != 1 or target.dtype not in (torch.int64, torch.int32):
        return False
    if input.dim() == 2:
        if input.dtype not in (torch.float32, torch.float64) or input.stride(1) != 1 or input.requires_grad:
            return False
        c = input.shape[1] if num_classes is None else num_classes
        if c != input.shape[1] or input.shape[0] != target.shape[0]:
            return False
    elif input.dim() == 1 and input.dtype in (torch.int64, torch.int32) and num_classes:
        c = num_classes
    else:
        return False
    # out-of-range labels take the ATen path, which raises the reference's own error
    return bool(native().cpu_labels_valid(input, target, int(c)))


def native_cls(
    input: torch.Tensor, target: torch.Tensor, *states: torch.Tensor, num_classes: Optional[int] = None
) -> bool:
    """True when (input, target) go through K1 (ROCm) or its host twin (small CPU batches with
    valid labels) and every destination state is float32."""
    if not all(s.dtype == torch.float32 and s.is_contiguous() for s in states):
        return False
    if input.is_cuda:
        return use_native(input) and target.is_cuda and cls_counts_supported(input, target)
    return _cpu_cls(input, target, num_classes)


_CPU_PRF_TARGETS = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)
_CPU_PRF_MAX = 1 << 16


def _cpu_prf_ok(input: torch.Tensor, target: torch.Tensor) -> bool:
    """Small 1-D CPU batches with integer / bool targets: binary precision / recall / F1 in one
    host call (csrc/runtime/cpu_metrics.cpp cpu_binary_prf) instead of ~10 ATen dispatches.
    Float targets keep the ATen path (its float sums and its bitwise-op errors)."""
    return (
        input.device.type == "cpu"
        and target.device.type == "cpu"
        and input.dim() == 1
        and target.dim() == 1
        and input.shape == target.shape
        and input.dtype in (torch.float32, torch.float64)
        and target.dtype in _CPU_PRF_TARGETS
        and input.numel() <= _CPU_PRF_MAX
        and not input.requires_grad
        and not compiling()
        and native_loaded()
    )


_AVERAGES = {"macro": 0, "weighted": 1}


def cpu_class_average(kind: int, average, a: torch.Tensor, b: torch.Tensor, c: Optional[torch.Tensor] = None):
    """Macro / weighted averages of small CPU float32 per-class count vectors in one host call
    (csrc/runtime/cpu_metrics.cpp cpu_class_average) instead of the ~10-op ATen mask / divide /
    nan_to_num / mean chain.  kind: 0 accuracy (correct, total), 1 F1 (tp, label, pred),
    2 precision (tp, fp, label), 3 recall (tp, label, pred).  Returns (0-d float32 value, some
    class has no label, recall's NaN class positions) or None (take the ATen path)."""
    if average not in _AVERAGES or (kind == 0 and average != "macro"):
        return None
    if compiling() or _ops.DISABLE_HIP or not native_loaded() or a.numel() > _CPU_MAX:
        return None
    for v in (a, b) if c is None else (a, b, c):
        if (v.device.type != "cpu" or v.dtype != torch.float32 or v.dim() != 1 or not v.is_contiguous()
                or v.numel() != a.numel() or v.requires_grad):
            return None
    return native().cpu_class_average(kind, _AVERAGES[average], a, b, c)


def cpu_class_metric(kind: int, average, input: torch.Tensor, target: torch.Tensor,
                     num_classes: Optional[int], k: int = 1):
    """A whole macro / weighted multiclass functional (kinds as ``cpu_class_average``) of a small
    CPU batch in one host call: class histograms and the average.  Returns the
    ``cpu_class_average`` triple, or None (other shapes / dtypes / devices, or a label out of
    range: the caller's ATen path then runs and raises the reference's errors)."""
    if average not in _AVERAGES or (kind == 0 and average != "macro"):
        return None
    if compiling() or _ops.DISABLE_HIP or input.is_cuda or target.is_cuda or not native_loaded():
        return None
    if type(num_classes) is not int or num_classes <= 0 or input.numel() > _CPU_MAX or input.requires_grad:
        return None
    if target.dim() != 1 or target.dtype not in (torch.int64, torch.int32) or input.shape[0] != target.shape[0]:
        return None
    if input.dim() == 2:
        if input.dtype not in (torch.float32, torch.float64) or input.shape[1] != num_classes or input.stride(1) != 1:
            return None
    elif input.dim() != 1 or input.dtype not in (torch.int64, torch.int32) or k != 1:
        return None
    return native().cpu_class_metric(kind, _AVERAGES[average], input, target, num_classes, k)


def cpu_confusion(input: torch.Tensor, target: torch.Tensor, num_classes: int, threshold: float = 0.5,
                  binary: bool = False) -> Optional[torch.Tensor]:
    """[C, C] confusion counts of a small CPU batch in one host call (the target's integer dtype,
    as the reference's ``ones_like(target)`` sparse sum), or None: out-of-range labels, other
    dtypes / devices (the caller's checking path then runs)."""
    if compiling() or _ops.DISABLE_HIP or input.is_cuda or target.is_cuda or not native_loaded():
        return None
    if target.dim() != 1 or target.dtype not in (torch.int64, torch.int32) or input.numel() > _CPU_MAX:
        return None
    if input.shape[0] != target.shape[0] or input.shape[0] == 0 or input.requires_grad:
        return None  # (an empty batch takes the checking path: the reference's torch.max raises)
    if binary or input.dim() == 2:
        if input.dtype not in (torch.float32, torch.float64) or input.dim() != (1 if binary else 2):
            return None
        if not binary and (input.shape[1] != num_classes or input.stride(1) != 1):
            return None
    elif input.dim() != 1 or input.dtype not in (torch.int64, torch.int32):
        return None
    return native().cpu_confusion(input, target, int(num_classes), float(threshold), bool(binary))


def _f32_scalars(*states: torch.Tensor) -> bool:
    """0-d float32 CPU states (the host twins' in-place contract)."""
    return all(s.dim() == 0 and s.dtype == torch.float32 and s.device.type == "cpu" for s in states)


def native_binary(input: torch.Tensor, target: torch.Tensor, *states: torch.Tensor) -> bool:
    return (
        use_native(input)
        and target.is_cuda
        and input.dtype in _BINARY_DTYPES
        and target.dtype in _BINARY_DTYPES
        and all(s.dtype == torch.float32 and s.is_contiguous() for s in states)
    )


def cls_counts(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    k: int = 1,
    num_classes: int = 0,
    micro_correct: Optional[torch.Tensor] = None,
    micro_incorrect: Optional[torch.Tensor] = None,
    micro_total: Optional[torch.Tensor] = None,
    micro_total2: Optional[torch.Tensor] = None,
    cls_correct: Optional[torch.Tensor] = None,
    cls_label: Optional[torch.Tensor] = None,
    cls_pred: Optional[torch.Tensor] = None,
    cls_fp: Optional[torch.Tensor] = None,
    confusion: Optional[torch.Tensor] = None,
    err: Optional[torch.Tensor] = None,
) -> None:
    """Accumulate argmax / top-k correctness counts and class histograms in one pass.

    micro_*: scalars (correct rows, wrong rows, += N twice); cls_*: [num_classes]
    (correct at target, rows per target, rows per prediction, wrong rows per prediction);
    confusion: [num_classes, num_classes] indexed (target, prediction).
    """
    if not target.is_contiguous():
        target = target.contiguous()
    if input.dim() == 2 and num_classes <= 0:
        num_classes = input.shape[1]
    if compiling() and input.is_cuda:  # dispatcher op: visible to torch.compile
        if micro_incorrect is not None or micro_total2 is not None or cls_fp is not None:
            raise NotImplementedError("cls_counts under torch.compile: micro_incorrect / micro_total2 / "
                                      "cls_fp destinations are eager-only")
        torch.ops.torcheval_amd.cls_counts(input, target, int(k), int(num_classes), micro_correct, micro_total,
                                           cls_correct, cls_label, cls_pred, confusion, err)
        return
    op = native().cls_counts if input.is_cuda else native().cpu_cls_counts
    op(
        input,
        target,
        int(k),
        int(num_classes),
        micro_correct,
        micro_total,
        cls_correct,
        cls_label,
        cls_pred,
        confusion,
        err,
        MAX_BLOCKS,
        micro_incorrect,
        micro_total2,
        cls_fp,
    )


def binary_counts(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: float = 0.5,
    weight: Optional[torch.Tensor] = None,
    tp: Optional[torch.Tensor] = None,
    fp: Optional[torch.Tensor] = None,
    tn: Optional[torch.Tensor] = None,
    fn: Optional[torch.Tensor] = None,
    total: Optional[torch.Tensor] = None,
    tp2: Optional[torch.Tensor] = None,
    fp2: Optional[torch.Tensor] = None,
    tn2: Optional[torch.Tensor] = None,
    fn2: Optional[torch.Tensor] = None,
    strict: bool = False,
) -> None:
    """Accumulate thresholded binary confusion counts in one pass.

    pred = ``input >= threshold``; tp/fp/tn/fn (optionally weighted) are added to each given
    destination and to its optional second destination (``*2``); ``total`` += N.  With
    ``strict`` a target outside {0, 1} counts nowhere; otherwise it is a wrong prediction.
    """
    if compiling() and tp2 is None and fp2 is None and tn2 is None and fn2 is None:
        # the dispatcher op (Meta kernel) keeps a compiled update in one graph
        torch.ops.torcheval_amd.binary_counts(input, target, weight, float(threshold), tp, fp, tn, fn, total,
                                              int(strict))
        return
    native().binary_counts(
        input, target, weight, float(threshold), tp, fp, tn, fn, total, int(strict), MAX_BLOCKS,
        tp2, fp2, tn2, fn2,
    )


# ----------------------------------------------------------------------------- K2 multilabel
_ML_SCORE = (torch.float32, torch.bfloat16, torch.float16)
_ML_TARGET = (torch.float32, torch.int64, torch.int32, torch.uint8, torch.bool)
ML_CRITERIA = {"exact_match": 0, "hamming": 1, "overlap": 2, "contain": 3, "belong": 4}
ML_MAX_TOPK_COLS = 2048


def native_multilabel(input: torch.Tensor, target: torch.Tensor, k: int = 0) -> bool:
    """True when (input, target) can go through K2 (``k > 0``: top-k mode)."""
    return (
        use_native(input)
        and target.is_cuda
        and input.dim() == 2
        and input.shape == target.shape
        and input.dtype in _ML_SCORE
        and target.dtype in _ML_TARGET
        and input.stride(1) == 1
        and target.stride(1) == 1
        and (k == 0 or input.shape[1] <= ML_MAX_TOPK_COLS)
        and input.numel() < 2**31
    )


def multilabel_counts(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    threshold: float,
    k: int,
    criteria: str,
    num_correct: torch.Tensor,
    num_total: "torch.Tensor | None" = None,
) -> None:
    """K2: add the update's correct count (and total) into float32 scalar states."""
    total = float(target.numel() if criteria == "hamming" else target.shape[0])
    _ml = torch.ops.torcheval_amd.multilabel_counts if compiling() else native().multilabel_counts
    _ml(
        input, target, float(threshold), int(k), ML_CRITERIA[criteria], num_correct, num_total, total
    )
