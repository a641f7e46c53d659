"""Precision, class API (parity: classification/precision.py:25-250).

GPU update = ONE K1 launch accumulating into the states; states are ``merge="sum"``.
"""

from typing import Iterable, Optional, TypeVar

import torch

from torcheval_amd.metrics.functional.classification.precision import (
    _binary_precision_update,
    _precision_compute,
    _precision_param_check,
    _precision_update,
    _precision_update_input_check,
)
from torcheval_amd.metrics.metric import Metric, inference_update
from torcheval_amd.ops import native
from torcheval_amd.ops.classification import _cpu_prf_ok, _f32_scalars, cls_counts, native_cls

TPrecision = TypeVar("TPrecision")
TBinaryPrecision = TypeVar("TBinaryPrecision")


class MulticlassPrecision(Metric[torch.Tensor]):
    """
    Precision for ``[N]`` labels or ``[N, C]`` scores.

    Args:
        num_classes: required unless ``average="micro"``.
        average: ``"micro"`` (default) | ``"macro"`` | ``"weighted"`` | ``None``.
    Functional version: ``torcheval_amd.metrics.functional.multiclass_precision``.
    """

    _err_words = 1  # K1 device flag: one int32 code

    def __init__(
        self: TPrecision,
        *,
        num_classes: Optional[int] = None,
        average: Optional[str] = "micro",
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _precision_param_check(num_classes, average)
        self.num_classes = num_classes
        self.average = average
        self._err: Optional[torch.Tensor] = None
        shape = () if average == "micro" else (num_classes,)
        for name in ("num_tp", "num_fp", "num_label"):
            self._add_state(name, torch.zeros(shape, device=self.device), merge="sum")

    def update(self: TPrecision, input: torch.Tensor, target: torch.Tensor) -> TPrecision:
        """Update states with predictions (``[N]`` or ``[N, C]``) and ``[N]`` targets."""
        input = input.to(self.device)
        target = target.to(self.device)
        if native_cls(input, target, self.num_tp, self.num_fp, self.num_label):
            _precision_update_input_check(input, target, self.num_classes)
            if self.average == "micro":
                cls_counts(input, target, micro_correct=self.num_tp, micro_incorrect=self.num_fp)
            else:
                if self._err is None:
                    self._err = torch.zeros(1, dtype=torch.int32, device=input.device)
                cls_counts(input, target, num_classes=self.num_classes, cls_correct=self.num_tp,
                           cls_fp=self.num_fp, cls_label=self.num_label, err=self._err)
            return self
        with torch.inference_mode():
            num_tp, num_fp, num_label = _precision_update(
                input, target, self.num_classes, self.average
            )
            self.num_tp += num_tp
            self.num_fp += num_fp
            self.num_label += num_label
        return self

    @torch.inference_mode()
    def compute(self: TPrecision) -> torch.Tensor:
        """Return the precision (0 for classes with neither predictions nor labels)."""
        from torcheval_amd.metrics.classification.accuracy import _raise_on_device_error

        _raise_on_device_error(self._err)
        return _precision_compute(self.num_tp, self.num_fp, self.num_label, self.average)

    @torch.inference_mode()
    def merge_state(self: TPrecision, metrics: Iterable[TPrecision]) -> TPrecision:
        for metric in metrics:
            self.num_tp += metric.num_tp.to(self.device)
            self.num_fp += metric.num_fp.to(self.device)
            self.num_label += metric.num_label.to(self.device)
        return self


class BinaryPrecision(MulticlassPrecision):
    """Precision of thresholded ``input`` (``input >= threshold`` is positive).
    Functional version: ``torcheval_amd.metrics.functional.binary_precision``."""

    _err_words = 0  # ATen update: no device flag

    def __init__(
        self: TBinaryPrecision,
        *,
        threshold: float = 0.5,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(num_classes=2, device=device)
        self.threshold = threshold

    @inference_update
    def update(self: TBinaryPrecision, input: torch.Tensor, target: torch.Tensor) -> TBinaryPrecision:
        """Update states with ``[N]`` scores and ``[N]`` binary targets."""
        input = input.to(self.device)
        target = target.to(self.device)
        if _cpu_prf_ok(input, target) and _f32_scalars(self.num_tp, self.num_fp):
            native().cpu_binary_prf_update(input, target, float(self.threshold), 0, self.num_tp, self.num_fp)
            return self
        num_tp, num_fp, num_label = _binary_precision_update(input, target, self.threshold)
        self.num_tp += num_tp
        self.num_fp += num_fp
        self.num_label += num_label
        return self
