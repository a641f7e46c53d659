"""Confusion matrix, class API (parity: classification/confusion_matrix.py:26-282).

GPU update = one K1 launch scattering into the [C, C] float state (no host sync: label
validation is a device flag checked at ``compute()``).  The state is ``merge="sum"``, so
``sync_and_compute`` of C=1000 is one 4 MB RCCL all-reduce.
"""

from typing import Iterable, Optional, TypeVar

import torch

from torcheval_amd.metrics.functional.classification.confusion_matrix import (
    _binary_confusion_matrix_update,
    _confusion_matrix_compute,
    _confusion_matrix_param_check,
    _confusion_matrix_shape_check,
    _confusion_matrix_update,
    _raise_confusion_err,
)
from torcheval_amd.metrics.metric import Metric, inference_update
from torcheval_amd.ops.classification import cls_counts, native_cls
from torcheval_amd.ops.hostread import read_ints

TMulticlassConfusionMatrix = TypeVar("TMulticlassConfusionMatrix")
TBinaryConfusionMatrix = TypeVar("TBinaryConfusionMatrix")


class MulticlassConfusionMatrix(Metric[torch.Tensor]):
    """
    [C, C] confusion matrix (row = target, column = prediction).

    Args:
        num_classes: number of classes (>= 2).
        normalize: None | "none" | "true" (rows) | "pred" (columns) | "all".
    Functional version: ``multiclass_confusion_matrix``.
    """

    _err_words = 3  # [flags, max bad target, max bad prediction]

    def __init__(
        self: TMulticlassConfusionMatrix,
        num_classes: int,
        *,
        normalize: Optional[str] = None,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _confusion_matrix_param_check(num_classes, normalize)
        self.normalize = normalize
        self.num_classes = num_classes
        # GPU updates: [flags, max bad target, max bad prediction] (int32, on device), and the
        # dtypes the error message prints them with
        self._err: Optional[torch.Tensor] = None
        self._err_dtypes = (torch.int64, torch.int64)
        self._add_state(
            "confusion_matrix",
            torch.zeros([num_classes, num_classes], device=self.device),
            merge="sum",
        )

    def update(
        self: TMulticlassConfusionMatrix, input: torch.Tensor, target: torch.Tensor
    ) -> TMulticlassConfusionMatrix:
        input = input.to(self.device)
        target = target.to(self.device)
        if native_cls(input, target, self.confusion_matrix, num_classes=self.num_classes) and input.shape[0] > 0:
            _confusion_matrix_shape_check(input, target, self.num_classes)
            if not input.is_cuda:  # the host twin ran after a label-range check: nothing to flag
                cls_counts(input, target, num_classes=self.num_classes, confusion=self.confusion_matrix.view(-1))
                return self
            if self._err is None:
                self._err = torch.zeros(3, dtype=torch.int32, device=input.device)
            self._err_dtypes = (target.dtype, input.dtype)
            cls_counts(input, target, num_classes=self.num_classes,
                       confusion=self.confusion_matrix.view(-1), err=self._err)
            return self
        with torch.inference_mode():
            self.confusion_matrix += _confusion_matrix_update(input, target, self.num_classes)
        return self

    def _check_device_errors(self) -> None:
        if self._err is None:
            return
        code, max_t, max_p = read_ints(self._err)
        if code != 0:
            self._err.zero_()
            # same message as the reference's update-time check (its torch.max of the batch is
            # the largest offending value, which the kernel records)
            _raise_confusion_err(torch.tensor([code]), torch.tensor(max_p, dtype=self._err_dtypes[1]),
                                 torch.tensor(max_t, dtype=self._err_dtypes[0]), self.num_classes)

    def compute(self: TMulticlassConfusionMatrix) -> torch.Tensor:
        if self._err is None and self.normalize in (None, "none"):
            # the raw counts: no tensor op, so no inference-mode context (~2-4 us on small states)
            out = self.confusion_matrix
            return out.clone() if self._tea_sb is not None else out
        with torch.inference_mode():
            return self._compute()

    def _compute(self: TMulticlassConfusionMatrix) -> torch.Tensor:
        self._check_device_errors()
        out = _confusion_matrix_compute(self.confusion_matrix, normalize=self.normalize)
        # never hand out a state that lives in a state buffer: reset() restores it in place
        return out.clone() if out is self.confusion_matrix and self._tea_sb is not None else out

    @torch.inference_mode()
    def normalized(self: TMulticlassConfusionMatrix, normalize: Optional[str] = None) -> torch.Tensor:
        """The confusion matrix normalised with ``normalize`` (ignores the constructor's)."""
        _confusion_matrix_param_check(self.num_classes, normalize)
        self._check_device_errors()
        out = _confusion_matrix_compute(self.confusion_matrix, normalize)
        return out.clone() if out is self.confusion_matrix and self._tea_sb is not None else out

    @torch.inference_mode()
    def merge_state(
        self: TMulticlassConfusionMatrix, metrics: Iterable[TMulticlassConfusionMatrix]
    ) -> TMulticlassConfusionMatrix:
        for metric in metrics:
            self.confusion_matrix += metric.confusion_matrix.to(self.device)
        return self


class BinaryConfusionMatrix(MulticlassConfusionMatrix):
    """2x2 confusion matrix of thresholded ``input``.  Functional: ``binary_confusion_matrix``."""

    _err_words = 0  # ATen update: no device flag

    def __init__(
        self: TBinaryConfusionMatrix,
        *,
        threshold: float = 0.5,
        normalize: Optional[str] = None,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(num_classes=2, device=device, normalize=normalize)
        self.threshold = threshold

    @inference_update
    def update(
        self: TBinaryConfusionMatrix, input: torch.Tensor, target: torch.Tensor
    ) -> TBinaryConfusionMatrix:
        input = input.to(self.device)
        target = target.to(self.device)
        self.confusion_matrix += _binary_confusion_matrix_update(input, target, self.threshold)
        return self
