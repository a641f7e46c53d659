"""ClickThroughRate class metric (parity: metrics/ranking/click_through_rate.py)."""

from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.ranking import (
    _click_through_rate_compute,
    _click_through_rate_input_check,
    _click_through_rate_update,
)
from torcheval_amd.metrics._pending import PendingMixin, RowSumsSpec, pending_states
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

__all__ = ["ClickThroughRate"]

_NAMES = ("click_total", "weight_total")
_CODES = (_rs.code(_rs.WX, _rs.ADD), _rs.code(_rs.W, _rs.ADD))


@pending_states(*_NAMES)
class ClickThroughRate(PendingMixin, Metric[torch.Tensor]):
    """Weighted click-through rate per task (float64 sums, ``merge="sum"``).

    ROCm batches whose task rows exceed 32K samples run K5b in deferred mode
    (metrics/_pending.py): block partials go to pending slots, folded when the states are read."""

    def __init__(self, *, num_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        if num_tasks < 1:
            raise ValueError(
                "`num_tasks` value should be greater than and equal to 1, but received {num_tasks}. "
            )
        self.num_tasks = num_tasks
        for name in ("click_total", "weight_total"):
            self._add_state(name, torch.zeros(num_tasks, dtype=torch.float64, device=self.device), merge="sum")

    def update(self, input: torch.Tensor, weights: Union[torch.Tensor, float, int] = 1.0) -> "ClickThroughRate":
        ct, wt = (self._raw_state(n) for n in _NAMES)  # no fold: an update only adds
        tw = isinstance(weights, torch.Tensor)
        if _rs.weight_ok(input, weights) and _rs.supported(input, weights if tw else None, states=(ct, wt)):
            _click_through_rate_input_check(input, weights, num_tasks=self.num_tasks)
            w, wsc = (weights, 1.0) if tw else (None, float(weights))
            if self._rowsums_deferred(input, w, wsc, RowSumsSpec(_NAMES, _CODES, self.num_tasks)):
                return self
            _rs.update(input, None, w, wsc, [ct, wt], list(_CODES), self.num_tasks)
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            click_total, weight_total = _click_through_rate_update(input, weights, num_tasks=self.num_tasks)
            self.click_total = self.click_total + click_total
            self.weight_total = self.weight_total + weight_total
            return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _click_through_rate_compute(self.click_total, self.weight_total)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["ClickThroughRate"]) -> "ClickThroughRate":
        for metric in metrics:
            self.click_total = self.click_total + metric.click_total.to(self.device)
            self.weight_total = self.weight_total + metric.weight_total.to(self.device)
        return self
