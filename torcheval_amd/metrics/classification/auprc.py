"""AUPRC, class API (parity: classification/auprc.py:31-420)."""

from typing import Optional

import torch

from torcheval_amd.metrics.classification._sample_store import SampleStoreMetric
from torcheval_amd.metrics.functional.classification.auprc import (
    _binary_auprc_compute,
    _binary_auprc_update_input_check,
    _multiclass_auprc_compute,
    _multiclass_auprc_param_check,
    _multiclass_auprc_update_input_check,
    _multilabel_auprc_compute,
    _multilabel_auprc_param_check,
    _multilabel_auprc_update_input_check,
)


class BinaryAUPRC(SampleStoreMetric[torch.Tensor]):
    """Area under the PR curve of ``[n]`` / ``[num_tasks, n]`` scores.
    Functional version: ``binary_auprc``."""

    _cat_dim = -1

    def __init__(self, *, num_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        if num_tasks < 1:
            raise ValueError("`num_tasks` must be an integer greater than or equal to 1")
        self.num_tasks = num_tasks

    def _check(self, input, target) -> None:
        _binary_auprc_update_input_check(input, target, self.num_tasks)

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        """Return the AUPRC (per task when ``num_tasks > 1``)."""
        return _binary_auprc_compute(*self._cat(), self.num_tasks)


class MulticlassAUPRC(SampleStoreMetric[torch.Tensor]):
    """One-vs-rest AUPRC of ``[n, C]`` scores; ``average`` in macro | None.
    Functional version: ``multiclass_auprc``."""

    def __init__(
        self, *, num_classes: int, average: Optional[str] = "macro", device: Optional[torch.device] = None
    ) -> None:
        super().__init__(device=device)
        _multiclass_auprc_param_check(num_classes, average)
        self.num_classes = num_classes
        self.average = average

    def _check(self, input, target) -> None:
        _multiclass_auprc_update_input_check(input, target, self.num_classes)

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _multiclass_auprc_compute(*self._cat(), self.average, self.num_classes)


class MultilabelAUPRC(SampleStoreMetric[torch.Tensor]):
    """Per-label AUPRC of ``[n, L]`` scores; ``average`` in macro | None.
    Functional version: ``multilabel_auprc``."""

    def __init__(
        self, *, num_labels: int, average: Optional[str] = "macro", device: Optional[torch.device] = None
    ) -> None:
        super().__init__(device=device)
        _multilabel_auprc_param_check(num_labels, average)
        self.num_labels = num_labels
        self.average = average

    def _check(self, input, target) -> None:
        _multilabel_auprc_update_input_check(input, target, self.num_labels)

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _multilabel_auprc_compute(*self._cat(), self.num_labels, self.average)
