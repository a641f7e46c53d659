"""AUROC, class API (parity: classification/auroc.py:34-235).

Samples are kept on device as list states (``merge="cat"``: the distributed toolkit
all-gathers them over RCCL without pickling).  Unweighted updates store an empty placeholder
instead of the reference's float64 ones per sample (auroc.py:112-113), saving 8 B/sample of
HBM and sync traffic; placeholders are expanded only if some update was weighted.
"""

from typing import Iterable, List, Optional, TypeVar

import torch

from torcheval_amd.metrics.functional.classification.auroc import (
    _binary_auroc_compute,
    _binary_auroc_update_input_check,
    _multiclass_auroc_compute,
    _multiclass_auroc_param_check,
    _multiclass_auroc_update_input_check,
)
from torcheval_amd.metrics.functional.classification._curve import merged_areas, runs_mergeable, sort_run
from torcheval_amd.metrics.metric import Metric, inference_update

TAUROC = TypeVar("TAUROC")
TMulticlassAUROC = TypeVar("TMulticlassAUROC")


_NO_WEIGHT = {}


def _no_weight(device: torch.device) -> torch.Tensor:
    """The shared empty float64 placeholder of an unweighted batch (one per device, a normal
    tensor even when first made inside inference mode): no allocation per append."""
    t = _NO_WEIGHT.get(device)
    if t is None:
        with torch.inference_mode(False):
            t = _NO_WEIGHT[device] = torch.empty(0, dtype=torch.float64, device=device)
    return t


def _cat_weights(inputs: List[torch.Tensor], weights: List[torch.Tensor]) -> Optional[torch.Tensor]:
    if all(w.numel() == 0 for w in weights):
        return None
    full = [w if w.numel() else torch.ones_like(x, dtype=torch.float64) for x, w in zip(inputs, weights)]
    return torch.cat(full, -1)


class BinaryAUROC(Metric[torch.Tensor]):
    """
    Area under the ROC curve for ``[n]`` or ``[num_tasks, n]`` scores with optional
    per-sample weights.  Functional version: ``binary_auroc``.
    """

    def __init__(
        self: TAUROC,
        *,
        num_tasks: int = 1,
        device: Optional[torch.device] = None,
        use_fbgemm: Optional[bool] = False,
    ) -> None:
        super().__init__(device=device)
        if num_tasks < 1:
            raise ValueError(
                "`num_tasks` value should be greater than or equal to 1, but received {num_tasks}. "
            )
        self.num_tasks = num_tasks
        self.use_fbgemm = use_fbgemm
        self._add_state("inputs", [], merge="cat")
        self._add_state("targets", [], merge="cat")
        self._add_state("weights", [], merge="cat")

    def update(
        self: TAUROC,
        input: torch.Tensor,
        target: torch.Tensor,
        weight: Optional[torch.Tensor] = None,
    ) -> TAUROC:
        """Append a batch of scores, {0,1} targets and optional weights."""
        dev = self._device
        if input.device != dev or target.device != dev or (weight is not None and weight.device != dev):
            return self._update_moved(input, target, weight)
        # on the metric's device already: stored as they are (the reference's no-op ``.to``),
        # with no inference-mode context (see SampleStoreMetric.update)
        _binary_auroc_update_input_check(input, target, self.num_tasks, weight)
        self._sorted_runs = False
        self.inputs.append(input)
        self.targets.append(target)
        self.weights.append(weight if weight is not None else _no_weight(dev))
        return self

    @inference_update
    def _update_moved(self: TAUROC, input, target, weight) -> TAUROC:
        input = input.to(self._device)
        target = target.to(self._device)
        if weight is not None:
            weight = weight.to(self._device)
        _binary_auroc_update_input_check(input, target, self.num_tasks, weight)
        self._sorted_runs = False
        self.inputs.append(input)
        self.targets.append(target)
        self.weights.append(weight if weight is not None else _no_weight(self._device))
        return self

    @torch.inference_mode()
    def compute(self: TAUROC) -> torch.Tensor:
        """Return the AUROC (float64; per task when ``num_tasks > 1``)."""
        if self.num_tasks == 1 and runs_mergeable(self, self.inputs):
            # after a distributed sync: every rank shipped its samples as one sorted run
            w = None
            if any(v.numel() for v in self.weights):
                w = [v if v.numel() else torch.ones_like(x, dtype=torch.float64) for x, v in zip(self.inputs, self.weights)]
            roc, _ = merged_areas(self.inputs, self.targets, w, roc=True, pr=False)
            return roc[0]
        inputs = torch.cat(self.inputs, -1)
        targets = torch.cat(self.targets, -1)
        return _binary_auroc_compute(inputs, targets, _cat_weights(self.inputs, self.weights), self.use_fbgemm)

    @torch.inference_mode()
    def merge_state(self: TAUROC, metrics: Iterable[TAUROC]) -> TAUROC:
        self._sorted_runs = False
        for metric in metrics:
            if metric.inputs:
                self.inputs.append(torch.cat(metric.inputs, -1).to(self.device))
                self.targets.append(torch.cat(metric.targets, -1).to(self.device))
                w = _cat_weights(metric.inputs, metric.weights)
                self.weights.append(
                    w.to(self.device) if w is not None else self.inputs[-1].new_empty(0, dtype=torch.float64)
                )
        return self

    def reset(self: TAUROC) -> TAUROC:
        super().reset()
        self._sorted_runs = False
        return self

    def load_state_dict(self, state_dict, strict: bool = True) -> None:
        super().load_state_dict(state_dict, strict)
        self._sorted_runs = False  # loaded lists carry no ordering guarantee

    @torch.inference_mode()
    def _prepare_for_merge_state(self: TAUROC) -> None:
        if not self.inputs and self.num_tasks == 1:
            self._sorted_runs = True  # nothing to ship: trivially a (zero) sorted run
        if self.inputs and self.targets:
            w = _cat_weights(self.inputs, self.weights)
            self.inputs = [torch.cat(self.inputs, -1)]
            self.targets = [torch.cat(self.targets, -1)]
            self.weights = [w if w is not None else self.inputs[0].new_empty(0, dtype=torch.float64)]
            if self.num_tasks == 1 and self.inputs[0].dim() == 1 and self.inputs[0].dtype == torch.float32:
                # ship a sorted run: the synced metric merges runs instead of sorting the union
                s, t, ws = sort_run(self.inputs[0], self.targets[0], w)
                self.inputs, self.targets = [s], [t]
                self.weights = [ws if ws is not None else s.new_empty(0, dtype=torch.float64)]
                self._sorted_runs = True


class MulticlassAUROC(Metric[torch.Tensor]):
    """One-vs-rest AUROC of ``[n, C]`` scores; ``average`` in macro | None.
    Functional version: ``multiclass_auroc``."""

    def __init__(
        self: TMulticlassAUROC,
        *,
        num_classes: int,
        average: Optional[str] = "macro",
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        _multiclass_auroc_param_check(num_classes, average)
        self.num_classes = num_classes
        self.average = average
        self._add_state("inputs", [], merge="cat")
        self._add_state("targets", [], merge="cat")

    @inference_update
    def update(self: TMulticlassAUROC, input: torch.Tensor, target: torch.Tensor) -> TMulticlassAUROC:
        input = input.to(self.device)
        target = target.to(self.device)
        _multiclass_auroc_update_input_check(input, target, self.num_classes)
        self.inputs.append(input)
        self.targets.append(target)
        return self

    @torch.inference_mode()
    def compute(self: TMulticlassAUROC) -> torch.Tensor:
        return _multiclass_auroc_compute(
            torch.cat(self.inputs), torch.cat(self.targets), self.num_classes, self.average
        )

    @torch.inference_mode()
    def merge_state(self: TMulticlassAUROC, metrics: Iterable[TMulticlassAUROC]) -> TMulticlassAUROC:
        for metric in metrics:
            if metric.inputs:
                self.inputs.append(torch.cat(metric.inputs).to(self.device))
                self.targets.append(torch.cat(metric.targets).to(self.device))
        return self

    @torch.inference_mode()
    def _prepare_for_merge_state(self: TMulticlassAUROC) -> None:
        if self.inputs and self.targets:
            self.inputs = [torch.cat(self.inputs)]
            self.targets = [torch.cat(self.targets)]
