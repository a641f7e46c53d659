"""Accuracy family, class API.

Parity: torcheval/metrics/classification/accuracy.py (MulticlassAccuracy :32,
BinaryAccuracy :151, MultilabelAccuracy :215, TopKMultilabelAccuracy :317).

Hot path (the north-star benchmark): on a ROCm device ``MulticlassAccuracy.update`` is ONE
launch of the fused K1 kernel that atomically accumulates straight into the
``num_correct`` / ``num_total`` state tensors — no argmax/eq/sum temporaries, no
``torch.tensor(N)`` host allocation (reference accuracy.py:271), no host sync.  All states
are declared ``merge="sum"`` so ``sync_and_compute`` is a single RCCL all-reduce.
"""

from typing import Iterable, Optional, TypeVar

import torch

from torcheval_amd.metrics.functional.classification.accuracy import (
    _CPU_FAST_MAX,
    _accuracy_compute,
    _accuracy_param_check,
    _accuracy_update_input_check,
    _binary_accuracy_update,
    _binary_accuracy_update_input_check,
    _multiclass_accuracy_update_aten,
    _multilabel_accuracy_param_check,
    _multilabel_accuracy_update,
    _multilabel_accuracy_update_input_check,
    _topk_multilabel_accuracy_param_check,
    _topk_multilabel_accuracy_update,
    _topk_multilabel_accuracy_update_input_check,
    _cpu_binary_ok,
    _cpu_fast_ok,
)
from torcheval_amd.metrics.metric import Metric, inference_update
import torcheval_amd.ops as _ops
from torcheval_amd.ops import compiling, native, native_loaded, use_native
from torcheval_amd.ops.hostread import read_int

# K1 micro-accuracy entry of the loaded extension (None when unbuilt); metrics built while
# ``torcheval_amd.ops.DISABLE_HIP`` is set do not use it (checked per metric, at construction)
_FAST_MICRO = getattr(_ops._C, "micro_accuracy_update", None) if native_loaded() else None
from torcheval_amd.ops.classification import (
    binary_counts,
    cls_counts,
    native_cls,
    multilabel_counts,
    native_multilabel,
)

TAccuracy = TypeVar("TAccuracy")
TBinaryAccuracy = TypeVar("TBinaryAccuracy")
TMultilabelAccuracy = TypeVar("TMultilabelAccuracy")
TTopKMultilabelAccuracy = TypeVar("TTopKMultilabelAccuracy")


def _micro_op_ok(input: torch.Tensor, target: torch.Tensor, state: torch.Tensor, num_classes: int) -> bool:
    """The preconditions ``_C.micro_accuracy_update`` tests itself, on metadata only (the
    torch.compile route: static under tracing, so the op is traced unconditionally)."""
    return (
        input.is_cuda
        and input.dim() == 2
        and target.dim() == 1
        and input.shape[0] == target.shape[0]
        and input.shape[1] > 0
        and (num_classes == 0 or input.shape[1] == num_classes)
        and input.stride(1) == 1
        and input.dtype in (torch.float32, torch.bfloat16, torch.float16)
        and target.dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)
        and target.is_contiguous()
        and target.device == input.device
        and state.device == input.device
    )


def _raise_on_device_error(err: Optional[torch.Tensor]) -> None:
    """Surface a device-side validation failure recorded by a K1 kernel."""
    code = read_int(err) if err is not None else 0
    if code != 0:
        err.zero_()
        raise RuntimeError(
            "index out of bounds: a target (or predicted) class index was outside "
            f"[0, num_classes) in an earlier update() (device error bits {code})."
        )


class MulticlassAccuracy(Metric[torch.Tensor]):
    """
    Frequency of ``input`` (labels ``[N]`` or scores ``[N, C]``) matching ``target``.

    Args:
        average: ``"micro"`` (default), ``"macro"`` or ``None``/``"none"`` (per class).
        num_classes: required for ``"macro"`` / ``None``.
        k: a sample counts as correct if its target is among the top-``k`` scores.
    Functional version: ``torcheval_amd.metrics.functional.multiclass_accuracy``.
    """

    def __init__(
        self: TAccuracy,
        *,
        average: Optional[str] = "micro",
        num_classes: Optional[int] = None,
        k: int = 1,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _accuracy_param_check(average, num_classes, k)
        self.average = average
        self.num_classes = num_classes
        self.k = k
        self._err: Optional[torch.Tensor] = None
        # K1 micro kernel: correct counts of the launches since the last fold, in 64 int64
        # cells (one no-return atomic per wave, no grid-wide fold on the update's tail);
        # ``num_correct`` folds them in on its next read (compute, sync, state_dict, merge)
        self._pend: Optional[torch.Tensor] = None
        self._pend_id = 0
        self._pend_dirty = False
        shape = () if average == "micro" else (num_classes or 0,)
        self._add_state("num_correct", torch.zeros(shape, device=self.device), merge="sum")
        self._add_state("num_total", torch.zeros(shape, device=self.device), merge="sum")
        self._refresh_fast_path()

    @property
    def _err_words(self) -> int:
        # K1's device flag (one int32 code) exists only where the update validates labels:
        # micro k=1 never creates one, so its sync carries no flag slot and compute() no read
        return 0 if self.average == "micro" and self.k == 1 else 1

    def _refresh_fast_path(self) -> None:
        # north-star fast path (ROCm states, micro, k=1): ONE native call that tests every
        # precondition itself and returns False for anything it does not handle
        self._fast = (
            _FAST_MICRO is not None
            and not _ops.DISABLE_HIP
            and self.average == "micro"
            and self.k == 1
            and type(self) is MulticlassAccuracy
            and self._device.type == "cuda"
        )
        # the native call declines inputs whose class count differs from num_classes, so the
        # reference's shape ValueError is raised on the Python path (reference accuracy.py:340)
        self._fast_nc = self.num_classes or 0

    def to(self: TAccuracy, device, *args, **kwargs) -> TAccuracy:
        super().to(device, *args, **kwargs)  # reads (so folds) num_correct first
        self._pend = None
        self._refresh_fast_path()
        return self

    # -- num_correct with the deferred fold of the K1 micro kernel's pending cells
    # (the tensor lives under "_nc": an instance-dict key named like the property confuses
    # torch.compile's tracing of the property)
    def _get_num_correct(self) -> torch.Tensor:
        d = self.__dict__
        if d.get("_pend_dirty"):
            self._fold_pending()
        return d["_nc"]

    def _set_num_correct(self, value: torch.Tensor) -> None:
        d = self.__dict__
        if d.get("_pend_dirty"):  # the pending counts belong to the value being replaced
            d["_pend"].zero_()
            d["_pend_dirty"] = False
        d["_nc"] = value

    num_correct = property(_get_num_correct, _set_num_correct)

    def _fold_pending(self, out: Optional[torch.Tensor] = None) -> None:
        d = self.__dict__
        native().micro_accuracy_finish(d["_pend"], d["_nc"], d["num_total"], out)
        d["_pend_dirty"] = False

    def _mark_updated(self, captured=None) -> None:
        """Called after a HIP-graph replay of ``update`` (torcheval_amd.utils.graphs); the K1
        pending cells are a fixed set, folded whole, so the capture token is not needed."""
        if self.__dict__.get("_pend") is not None:
            self.__dict__["_pend_dirty"] = True

    def _raw_state(self, name: str) -> torch.Tensor:
        """A state without folding the pending cells (graph replays' state-pointer checks)."""
        return self.__dict__["_nc"] if name == "num_correct" else getattr(self, name)

    def __getstate__(self):
        # copies (copy / deepcopy / pickle) carry folded states and no pending cells
        d = self.__dict__
        if d.get("_pend_dirty"):
            self._fold_pending()
        state = dict(d)
        state["_pend"] = None
        state["_pend_dirty"] = False
        return state

    def __setstate__(self, state) -> None:
        self.__dict__.update(state)

    def reset(self: TAccuracy) -> TAccuracy:
        d = self.__dict__
        if d.get("_pend_dirty"):
            d["_pend"].zero_()
            d["_pend_dirty"] = False
        return super().reset()

    def update(self: TAccuracy, input: torch.Tensor, target: torch.Tensor) -> TAccuracy:
        """
        Update states with a batch of predictions (``[N]`` labels or ``[N, C]`` scores)
        and ``[N]`` ground-truth labels.
        """
        if self._fast:
            if not compiling():
                d = self.__dict__
                pend = d["_pend"]
                if pend is None or d["_pend_id"] != id(self):
                    pend = d["_pend"] = torch.zeros(512, dtype=torch.int64, device=self._device)
                    d["_pend_id"] = id(self)
                if _FAST_MICRO(input, target, d["_nc"], d["num_total"], self._fast_nc, pend):
                    d["_pend_dirty"] = True
                    return self
            elif _micro_op_ok(input, target, self.num_correct, self._fast_nc):
                torch.ops.torcheval_amd.micro_accuracy(input, target, self.num_correct, self.num_total)
                return self
        dev = self._device
        if input.device != dev:
            input = input.to(dev)
        if target.device != dev:
            target = target.to(dev)
        _accuracy_update_input_check(input, target, self.num_classes, self.k)
        if (
            self.average == "micro"
            and not input.is_cuda
            and input.numel() <= _CPU_FAST_MAX
            and self.num_correct.dtype == torch.float32
            and _cpu_fast_ok(input, target, self.k, None)
        ):
            # small CPU batches (BASELINE config 1 shape): one fused C++ call accumulates the
            # counts into the states instead of ~6 ATen dispatches
            native().cpu_micro_accuracy_update(input, target, self.k, self.num_correct, self.num_total)
            return self
        if native_cls(input, target, self.num_correct, self.num_total,
                      num_classes=None if self.average == "micro" else self.num_classes):
            if self.average == "micro":
                if self.k > 1 and self._err is None:
                    self._err = torch.zeros(1, dtype=torch.int32, device=dev)
                cls_counts(
                    input,
                    target,
                    k=self.k,
                    num_classes=input.shape[1] if input.ndim == 2 else 0,
                    micro_correct=self.num_correct,
                    micro_total=self.num_total,
                    err=self._err,
                )
            else:
                if self._err is None:
                    self._err = torch.zeros(1, dtype=torch.int32, device=dev)
                cls_counts(
                    input,
                    target,
                    k=self.k,
                    num_classes=self.num_classes,
                    cls_correct=self.num_correct,
                    cls_label=self.num_total,
                    err=self._err,
                )
            return self
        with torch.inference_mode():
            num_correct, num_total = _multiclass_accuracy_update_aten(
                input, target, self.average, self.num_classes, self.k
            )
            self.num_correct += num_correct
            self.num_total += num_total
        return self

    def _check_device_errors(self) -> None:
        _raise_on_device_error(self._err)

    def compute(self: TAccuracy) -> torch.Tensor:
        """Return the accuracy (NaN if ``update()`` was never called)."""
        # the division is enqueued before the flag read, so that read (a host sync) does not
        # hold the launch back.  The states never require grad, so no autograd graph is
        # recorded; the inference_mode context (~4 us of host time) is only entered for the
        # macro path's masked indexing.
        d = self.__dict__
        if d.get("_pend_dirty"):  # fold the pending cells and divide: one launch
            out = torch.empty((), dtype=torch.float32, device=d["num_total"].device)
            self._fold_pending(out)
        elif self.average == "micro" or self.average is None or self.average == "none":
            out = self.num_correct / self.num_total
        else:
            with torch.inference_mode():
                out = _accuracy_compute(self.num_correct, self.num_total, self.average)
        self._check_device_errors()
        return out

    @torch.inference_mode()
    def merge_state(self: TAccuracy, metrics: Iterable[TAccuracy]) -> TAccuracy:
        for metric in metrics:
            self.num_correct += metric.num_correct.to(self.device)
            self.num_total += metric.num_total.to(self.device)
        return self


class BinaryAccuracy(MulticlassAccuracy):
    """
    Frequency of thresholded ``input`` matching ``target``
    (``torch.where(input < threshold, 0, 1)``).
    Functional version: ``torcheval_amd.metrics.functional.binary_accuracy``.
    """

    _err_words = 0  # no device flag

    def __init__(
        self: TBinaryAccuracy,
        *,
        threshold: float = 0.5,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        self.threshold = threshold

    def update(self: TBinaryAccuracy, input: torch.Tensor, target: torch.Tensor) -> TBinaryAccuracy:
        """Update states with ``[N]`` scores/labels and ``[N]`` ground truth."""
        input = input.to(self.device)
        target = target.to(self.device)
        _binary_accuracy_update_input_check(input, target)
        if (
            _cpu_binary_ok(input, target)
            and self.num_correct.dtype == torch.float32
            and self.num_total.dtype == torch.float32
            and self.num_correct.dim() == 0
            and self.num_total.dim() == 0
        ):
            native().cpu_binary_accuracy_update(input, target, float(self.threshold), self.num_correct, self.num_total)
            return self
        if use_native(input) and self.num_correct.dtype == torch.float32:
            binary_counts(
                input,
                target,
                threshold=self.threshold,
                tp=self.num_correct,
                tn=self.num_correct,
                total=self.num_total,
            )
            return self
        with torch.inference_mode():
            num_correct, num_total = _binary_accuracy_update(input, target, self.threshold)
            self.num_correct += num_correct
            self.num_total += num_total
        return self


def _k2_state_ok(metric: Metric, input: torch.Tensor, target: torch.Tensor, k: int) -> bool:
    return (
        native_multilabel(input, target, k)
        and metric.num_correct.dtype == torch.float32
        and metric.num_total.dtype == torch.float32
        and metric.num_correct.numel() == 1
        and metric.num_total.numel() == 1
    )


class MultilabelAccuracy(MulticlassAccuracy):
    """
    Multilabel accuracy; ``criteria`` in ``exact_match`` (default) | ``hamming`` |
    ``overlap`` | ``contain`` | ``belong``.
    Functional version: ``torcheval_amd.metrics.functional.multilabel_accuracy``.
    """

    _err_words = 0  # no device flag

    def __init__(
        self: TMultilabelAccuracy,
        *,
        threshold: float = 0.5,
        criteria: str = "exact_match",
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _multilabel_accuracy_param_check(criteria)
        self.threshold = threshold
        self.criteria = criteria

    @inference_update
    def update(
        self: TMultilabelAccuracy, input: torch.Tensor, target: torch.Tensor
    ) -> TMultilabelAccuracy:
        """Update states with ``[N, L]`` scores/labels and ``[N, L]`` ground truth."""
        input = input.to(self.device)
        target = target.to(self.device)
        if _k2_state_ok(self, input, target, 0):
            _multilabel_accuracy_update_input_check(input, target)
            multilabel_counts(
                input, target, threshold=self.threshold, k=0, criteria=self.criteria,
                num_correct=self.num_correct, num_total=self.num_total,
            )
            return self
        num_correct, num_total = _multilabel_accuracy_update(
            input, target, self.threshold, self.criteria
        )
        self.num_correct += num_correct
        self.num_total += num_total
        return self


class TopKMultilabelAccuracy(MulticlassAccuracy):
    """
    Multilabel accuracy of the top-``k`` scores.  The default is ``k=2`` (the reference's
    default ``k=1`` always fails its own check, classification/accuracy.py:380).
    Functional version: ``torcheval_amd.metrics.functional.topk_multilabel_accuracy``.
    """

    _err_words = 0  # no device flag

    def __init__(
        self: TTopKMultilabelAccuracy,
        *,
        criteria: str = "exact_match",
        k: int = 2,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _topk_multilabel_accuracy_param_check(criteria, k)
        self.criteria = criteria
        self.k = k

    @inference_update
    def update(
        self: TTopKMultilabelAccuracy, input: torch.Tensor, target: torch.Tensor
    ) -> TTopKMultilabelAccuracy:
        """Update states with ``[N, L]`` scores and ``[N, L]`` ground truth."""
        input = input.to(self.device)
        target = target.to(self.device)
        if _k2_state_ok(self, input, target, self.k):
            _topk_multilabel_accuracy_update_input_check(input, target, self.k)
            multilabel_counts(
                input, target, threshold=0.5, k=self.k, criteria=self.criteria,
                num_correct=self.num_correct, num_total=self.num_total,
            )
            return self
        num_correct, num_total = _topk_multilabel_accuracy_update(
            input, target, self.criteria, self.k
        )
        self.num_correct += num_correct
        self.num_total += num_total
        return self
