"""Recall, class API (parity: classification/recall.py:26-250)."""

from typing import Iterable, Optional, TypeVar

import torch

from torcheval_amd.metrics.functional.classification.recall import (
    _binary_recall_compute,
    _binary_recall_update,
    _recall_compute,
    _recall_param_check,
    _recall_update,
    _recall_update_input_check,
)
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import native
from torcheval_amd.ops.classification import _cpu_prf_ok, _f32_scalars, binary_counts, cls_counts, native_binary, native_cls

TBinaryRecall = TypeVar("TBinaryRecall")
TRecall = TypeVar("TRecall")


class BinaryRecall(Metric[torch.Tensor]):
    """Recall of thresholded ``input``.  Functional: ``binary_recall``."""

    def __init__(self: TBinaryRecall, *, threshold: float = 0.5, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self.threshold = threshold
        self._add_state("num_tp", torch.tensor(0.0, device=self.device), merge="sum")
        self._add_state("num_true_labels", torch.tensor(0.0, device=self.device), merge="sum")

    def update(self: TBinaryRecall, input: torch.Tensor, target: torch.Tensor) -> TBinaryRecall:
        """Update states with ``[N]`` scores and ``[N]`` integer/bool targets."""
        input = input.to(self.device)
        target = target.to(self.device)
        if (
            native_binary(input, target, self.num_tp, self.num_true_labels)
            and not target.is_floating_point()
            and input.shape == target.shape
            and target.ndim == 1
        ):
            binary_counts(input, target, threshold=self.threshold, tp=self.num_tp,
                          tp2=self.num_true_labels, fn=self.num_true_labels, strict=True)
            return self
        if _cpu_prf_ok(input, target) and _f32_scalars(self.num_tp, self.num_true_labels):
            native().cpu_binary_prf_update(input, target, float(self.threshold), 1, self.num_tp, self.num_true_labels)
            return self
        with torch.inference_mode():
            num_tp, num_true_labels = _binary_recall_update(input, target, self.threshold)
            self.num_tp += num_tp
            self.num_true_labels += num_true_labels
        return self

    @torch.inference_mode()
    def compute(self: TBinaryRecall) -> torch.Tensor:
        return _binary_recall_compute(self.num_tp, self.num_true_labels)

    @torch.inference_mode()
    def merge_state(self: TBinaryRecall, metrics: Iterable[TBinaryRecall]) -> TBinaryRecall:
        for metric in metrics:
            self.num_tp += metric.num_tp.to(self.device)
            self.num_true_labels += metric.num_true_labels.to(self.device)
        return self


class MulticlassRecall(Metric[torch.Tensor]):
    """
    Recall for ``[N]`` labels or ``[N, C]`` scores; ``average`` in micro | macro | weighted |
    None.  Functional version: ``multiclass_recall``.
    """

    _err_words = 1  # K1 device flag: one int32 code

    def __init__(
        self: TRecall,
        *,
        num_classes: Optional[int] = None,
        average: Optional[str] = "micro",
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _recall_param_check(num_classes, average)
        self.num_classes = num_classes
        self.average = average
        self._err: Optional[torch.Tensor] = None
        shape = () if average == "micro" else (num_classes,)
        for name in ("num_tp", "num_labels", "num_predictions"):
            self._add_state(name, torch.zeros(shape, device=self.device), merge="sum")

    def update(self: TRecall, input: torch.Tensor, target: torch.Tensor) -> TRecall:
        input = input.to(self.device)
        target = target.to(self.device)
        if native_cls(input, target, self.num_tp, self.num_labels, self.num_predictions):
            _recall_update_input_check(input, target, self.num_classes)
            if self.average == "micro":
                cls_counts(input, target, micro_correct=self.num_tp, micro_total=self.num_labels,
                           micro_total2=self.num_predictions)
            else:
                if self._err is None:
                    self._err = torch.zeros(1, dtype=torch.int32, device=input.device)
                cls_counts(input, target, num_classes=self.num_classes, cls_correct=self.num_tp,
                           cls_label=self.num_labels, cls_pred=self.num_predictions, err=self._err)
            return self
        with torch.inference_mode():
            num_tp, num_labels, num_predictions = _recall_update(
                input, target, self.num_classes, self.average
            )
            self.num_tp += num_tp
            self.num_labels += num_labels
            self.num_predictions += num_predictions
        return self

    def _check_device_errors(self) -> None:
        from torcheval_amd.metrics.classification.accuracy import _raise_on_device_error

        _raise_on_device_error(self._err)

    @torch.inference_mode()
    def compute(self: TRecall) -> torch.Tensor:
        self._check_device_errors()
        return _recall_compute(self.num_tp, self.num_labels, self.num_predictions, self.average)

    @torch.inference_mode()
    def merge_state(self: TRecall, metrics: Iterable[TRecall]) -> TRecall:
        for metric in metrics:
            self.num_tp += metric.num_tp.to(self.device)
            self.num_labels += metric.num_labels.to(self.device)
            self.num_predictions += metric.num_predictions.to(self.device)
        return self
