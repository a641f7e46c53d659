"""Shared base for metrics that keep every (input, target) sample until ``compute()``.

Reference pattern (auprc.py, precision_recall_curve.py, recall_at_fixed_precision.py,
binned_auroc.py): list states ``inputs`` / ``targets``, ``merge_state`` appends the other
metric's concatenation, ``_prepare_for_merge_state`` collapses the lists before a sync.
Here the lists are declared ``merge="cat"`` so the distributed toolkit moves them with one
device-resident all-gather-v over RCCL (no pickling), and samples never leave HBM.
"""

from typing import Iterable, TypeVar

import torch

from torcheval_amd.metrics.metric import Metric, TComputeReturn, inference_update

TSelf = TypeVar("TSelf", bound="SampleStoreMetric")


class SampleStoreMetric(Metric[TComputeReturn]):
    """Subclasses set ``_cat_dim`` and implement ``_check(input, target)`` / ``compute``."""

    _cat_dim: int = 0

    def __init__(self, *, device=None) -> None:
        super().__init__(device=device)
        self._add_state("inputs", [], merge="cat")
        self._add_state("targets", [], merge="cat")

    def _check(self, input: torch.Tensor, target: torch.Tensor) -> None:
        pass

    def update(self: TSelf, input: torch.Tensor, target: torch.Tensor) -> TSelf:
        """Append a batch of scores and targets (kept on the metric's device)."""
        dev = self._device
        if input.device != dev or target.device != dev:
            return self._update_moved(input, target)
        # already on the metric's device: the reference's ``.to`` is a no-op that stores the
        # caller's tensors themselves, so neither the copy nor the inference-mode context
        # (~2-4 us, the whole cost of a small append) is needed
        self._check(input, target)
        self.inputs.append(input)
        self.targets.append(target)
        return self

    @inference_update
    def _update_moved(self: TSelf, input: torch.Tensor, target: torch.Tensor) -> TSelf:
        input = input.to(self._device)
        target = target.to(self._device)
        self._check(input, target)
        self.inputs.append(input)
        self.targets.append(target)
        return self

    def _cat(self):
        return torch.cat(self.inputs, self._cat_dim), torch.cat(self.targets, self._cat_dim)

    @torch.inference_mode()
    def merge_state(self: TSelf, metrics: Iterable[TSelf]) -> TSelf:
        for metric in metrics:
            if metric.inputs:
                self.inputs.append(torch.cat(metric.inputs, self._cat_dim).to(self.device))
                self.targets.append(torch.cat(metric.targets, self._cat_dim).to(self.device))
        return self

    @torch.inference_mode()
    def _prepare_for_merge_state(self) -> None:
        if self.inputs and self.targets:
            self.inputs = [torch.cat(self.inputs, self._cat_dim)]
            self.targets = [torch.cat(self.targets, self._cat_dim)]
