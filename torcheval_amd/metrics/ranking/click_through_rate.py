"""ClickThroughRate class metric (parity: metrics/ranking/click_through_rate.py)."""

from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.ranking import (
    _click_through_rate_compute,
    _click_through_rate_input_check,
    _click_through_rate_update,
)
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

__all__ = ["ClickThroughRate"]


class ClickThroughRate(Metric[torch.Tensor]):
    """Weighted click-through rate per task (float64 sums, ``merge="sum"``)."""

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
        if _rs.weight_ok(input, weights) and _rs.supported(
            input, weights if isinstance(weights, torch.Tensor) else None, states=(self.click_total, self.weight_total)
        ):
            _click_through_rate_input_check(input, weights, num_tasks=self.num_tasks)
            _rs.update_states(input, None, weights, [(self.click_total, _rs.WX, _rs.ADD),
                                                     (self.weight_total, _rs.W, _rs.ADD)], rows=self.num_tasks)
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
