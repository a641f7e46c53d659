"""AUPRC, class API (parity: classification/auprc.py:31-420)."""

from typing import Optional

import torch

from torcheval_amd.metrics.classification._sample_store import SampleStoreMetric
from torcheval_amd.metrics.functional.classification._curve import merged_areas, runs_mergeable, sort_run
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

    def update(self, input: torch.Tensor, target: torch.Tensor) -> "BinaryAUPRC":
        self._sorted_runs = False
        return SampleStoreMetric.update(self, input, target)

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        """Return the AUPRC (per task when ``num_tasks > 1``)."""
        if self.num_tasks == 1 and runs_mergeable(self, self.inputs):
            _, pr = merged_areas(self.inputs, self.targets, None, roc=False, pr=True)  # synced sorted runs
            return pr[0].to(torch.float32)
        return _binary_auprc_compute(*self._cat(), self.num_tasks)

    @torch.inference_mode()
    def merge_state(self, metrics) -> "BinaryAUPRC":
        self._sorted_runs = False
        return super().merge_state(metrics)

    def reset(self) -> "BinaryAUPRC":
        super().reset()
        self._sorted_runs = False
        return self

    def load_state_dict(self, state_dict, strict: bool = True) -> None:
        super().load_state_dict(state_dict, strict)
        self._sorted_runs = False  # loaded lists carry no ordering guarantee

    @torch.inference_mode()
    def _prepare_for_merge_state(self) -> None:
        super()._prepare_for_merge_state()
        if not self.inputs and self.num_tasks == 1:
            self._sorted_runs = True  # nothing to ship: trivially a (zero) sorted run
        if self.num_tasks == 1 and self.inputs and self.inputs[0].dim() == 1 and self.inputs[0].dtype == torch.float32:
            s, t, _ = sort_run(self.inputs[0], self.targets[0], None)
            self.inputs, self.targets = [s], [t]
            self._sorted_runs = True


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
