"""Binned AUPRC class metrics on the K4 binned counts (parity: metrics/classification/binned_auprc.py)."""

from typing import List, Optional, Union

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.classification.binned_auprc import (
    _binary_binned_auprc_param_check,
    _binary_binned_auprc_update_input_check,
    _binned_riemann,
    _multiclass_binned_auprc_param_check,
    _multiclass_binned_auprc_update_input_check,
    _multilabel_binned_auprc_param_check,
    _multilabel_binned_auprc_update_input_check,
)
from torcheval_amd.metrics.functional.classification.binned_precision_recall_curve import (
    _optimization_param_check,
)
from torcheval_amd.metrics.functional.tensor_utils import _create_threshold_tensor
from torcheval_amd.metrics.classification.binned_precision_recall_curve import _BinnedCountsMetric

__all__ = ["BinaryBinnedAUPRC", "MulticlassBinnedAUPRC", "MultilabelBinnedAUPRC"]


class BinaryBinnedAUPRC(_BinnedCountsMetric):
    """Binned AUPRC of ``[n]`` / ``[num_tasks, n]`` scores (states [num_tasks, T]).
    Functional: ``binary_binned_auprc``."""

    def __init__(
        self,
        *,
        num_tasks: int = 1,
        threshold: Union[int, List[float], torch.Tensor] = 100,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        threshold = _create_threshold_tensor(threshold, self.device)
        _binary_binned_auprc_param_check(num_tasks, threshold)
        self.num_tasks = num_tasks
        self.threshold = threshold
        self._init_counts((num_tasks, len(threshold)))

    def _views(self):
        return self.num_tp.t(), self.num_fp.t(), self.num_fn.t()

    @inference_update
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "BinaryBinnedAUPRC":
        input = input.to(self.device)
        target = target.to(self.device)
        _binary_binned_auprc_update_input_check(input, target, self.num_tasks, self.threshold)
        if input.ndim == 1:
            input, target = input[None, :], target[None, :]
        self._accumulate(input.t(), target.t(), 0)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        auprc = _binned_riemann(self.num_tp.t(), self.num_fp.t(), self.num_fn.t())
        return auprc[0] if self.num_tasks == 1 else auprc


class MulticlassBinnedAUPRC(_BinnedCountsMetric):
    """One-vs-rest binned AUPRC.  Functional: ``multiclass_binned_auprc``."""

    def __init__(
        self,
        *,
        num_classes: int,
        threshold: Union[int, List[float], torch.Tensor] = 100,
        average: Optional[str] = "macro",
        optimization: str = "vectorized",
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _optimization_param_check(optimization)
        threshold = _create_threshold_tensor(threshold, self.device)
        _multiclass_binned_auprc_param_check(num_classes, threshold, average)
        self.num_classes = num_classes
        self.threshold = threshold
        self.average = average
        self.optimization = optimization
        self._init_counts((len(threshold), num_classes))

    @inference_update
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "MulticlassBinnedAUPRC":
        input = input.to(self.device)
        target = target.to(self.device)
        _multiclass_binned_auprc_update_input_check(input, target, self.num_classes)
        self._accumulate(input, target, 1)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        auprc = _binned_riemann(self.num_tp, self.num_fp, self.num_fn)
        return auprc.mean() if self.average == "macro" else auprc


class MultilabelBinnedAUPRC(_BinnedCountsMetric):
    """Per-label binned AUPRC.  Functional: ``multilabel_binned_auprc``."""

    def __init__(
        self,
        *,
        num_labels: int,
        threshold: Union[int, List[float], torch.Tensor] = 100,
        average: Optional[str] = "macro",
        optimization: str = "vectorized",
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _optimization_param_check(optimization)
        threshold = _create_threshold_tensor(threshold, self.device)
        _multilabel_binned_auprc_param_check(num_labels, threshold, average)
        self.num_labels = num_labels
        self.threshold = threshold
        self.average = average
        self.optimization = optimization
        self._init_counts((len(threshold), num_labels))

    @inference_update
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "MultilabelBinnedAUPRC":
        input = input.to(self.device)
        target = target.to(self.device)
        _multilabel_binned_auprc_update_input_check(input, target, self.num_labels)
        self._accumulate(input, target, 0)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        auprc = _binned_riemann(self.num_tp, self.num_fp, self.num_fn)
        return auprc.mean() if self.average == "macro" else auprc
