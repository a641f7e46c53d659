"""Recall at fixed precision, class API (parity: classification/recall_at_fixed_precision.py)."""

from typing import List, Optional, Tuple

import torch

from torcheval_amd.metrics.classification._sample_store import SampleStoreMetric
from torcheval_amd.metrics.functional.classification.recall_at_fixed_precision import (
    _binary_recall_at_fixed_precision_compute,
    _binary_recall_at_fixed_precision_update_input_check,
    _multilabel_recall_at_fixed_precision_compute,
    _multilabel_recall_at_fixed_precision_update_input_check,
)


class BinaryRecallAtFixedPrecision(SampleStoreMetric[Tuple[torch.Tensor, torch.Tensor]]):
    """(max recall with precision >= ``min_precision``, threshold).
    Functional: ``binary_recall_at_fixed_precision``."""

    def __init__(self, *, min_precision: float, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self.min_precision = min_precision

    def _check(self, input, target) -> None:
        _binary_recall_at_fixed_precision_update_input_check(input, target, self.min_precision)

    @torch.inference_mode()
    def compute(self) -> Tuple[torch.Tensor, torch.Tensor]:
        return _binary_recall_at_fixed_precision_compute(*self._cat(), self.min_precision)


class MultilabelRecallAtFixedPrecision(SampleStoreMetric[Tuple[List[torch.Tensor], List[torch.Tensor]]]):
    """Per-label (max recall, threshold).  Functional: ``multilabel_recall_at_fixed_precision``."""

    def __init__(self, *, num_labels: int, min_precision: float, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self.num_labels = num_labels
        self.min_precision = min_precision

    def _check(self, input, target) -> None:
        _multilabel_recall_at_fixed_precision_update_input_check(
            input, target, self.num_labels, self.min_precision
        )

    @torch.inference_mode()
    def compute(self) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
        return _multilabel_recall_at_fixed_precision_compute(*self._cat(), self.num_labels, self.min_precision)
