"""WeightedCalibration class metric (parity: metrics/ranking/weighted_calibration.py)."""

from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.ranking import _weighted_calibration_update
from torcheval_amd.metrics.functional.ranking._rank_common import _num_tasks_check
from torcheval_amd.metrics._pending import PendingMixin, RowSumsSpec, pending_states
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

__all__ = ["WeightedCalibration"]

_NAMES = ("weighted_input_sum", "weighted_target_sum")
_CODES = (_rs.code(_rs.WX, _rs.ADD), _rs.code(_rs.WT, _rs.ADD))


@pending_states(*_NAMES)
class WeightedCalibration(PendingMixin, Metric[torch.Tensor]):
    """sum(w * input) / sum(w * target) per task (float64 sums, ``merge="sum"``).

    ROCm batches whose task rows exceed 32K samples run K5b in deferred mode
    (metrics/_pending.py): block partials go to pending slots, folded when the states are read."""

    def __init__(self, *, num_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        if num_tasks < 1:
            raise ValueError(
                "`num_tasks` value should be greater than and equal to 1, but received {num_tasks}. "
            )
        self.num_tasks = num_tasks
        for name in ("weighted_input_sum", "weighted_target_sum"):
            self._add_state(name, torch.zeros(num_tasks, dtype=torch.float64, device=self.device), merge="sum")

    def update(
        self, input: torch.Tensor, target: torch.Tensor, weight: Union[float, int, torch.Tensor] = 1.0
    ) -> "WeightedCalibration":
        wi, wt = (self._raw_state(n) for n in _NAMES)  # no fold: an update only adds
        tw = isinstance(weight, torch.Tensor)
        if input.shape == target.shape and _rs.weight_ok(input, weight) and _rs.supported(
            input, target, weight if tw else None, states=(wi, wt)
        ):
            _num_tasks_check(input, self.num_tasks)
            w, wsc = (weight, 1.0) if tw else (None, float(weight))
            if self._rowsums_deferred(input, w, wsc, RowSumsSpec(_NAMES, _CODES, self.num_tasks), t=target):
                return self
            _rs.update(input, target, w, wsc, [wi, wt], list(_CODES), self.num_tasks)
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            wi, wt = _weighted_calibration_update(input, target, weight, num_tasks=self.num_tasks)
            self.weighted_input_sum += wi
            self.weighted_target_sum += wt
            return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if torch.any(self.weighted_target_sum == 0.0):
            return torch.empty(0)
        return self.weighted_input_sum / self.weighted_target_sum

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["WeightedCalibration"]) -> "WeightedCalibration":
        for metric in metrics:
            self.weighted_input_sum += metric.weighted_input_sum.to(self.device)
            self.weighted_target_sum += metric.weighted_target_sum.to(self.device)
        return self
