"""Sum class metric (parity: metrics/aggregation/sum.py)."""

from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.aggregation import _sum_update
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

__all__ = ["Sum"]

_CODES = [_rs.code(_rs.WX, _rs.ADD)]


class Sum(Metric[torch.Tensor]):
    """Weighted sum of all inputs (float64 accumulator)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("weighted_sum", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")

    def update(self, input: torch.Tensor, *, weight: Union[float, int, torch.Tensor] = 1.0) -> "Sum":
        if _rs.fast_ok(input, weight, self.weighted_sum):  # K5b, one launch (host twin on CPU)
            tw = isinstance(weight, torch.Tensor)
            _rs.update(input, None, weight if tw else None, 1.0 if tw else float(weight), [self.weighted_sum], _CODES)
            return self
        return self._update_aten(input, weight)

    @torch.inference_mode()
    def _update_aten(self, input: torch.Tensor, weight) -> "Sum":
        self.weighted_sum += _sum_update(input, weight)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        # a copy once the state lives in a state buffer: reset() then restores it in place
        return self.weighted_sum if self._tea_sb is None else self.weighted_sum.clone()

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Sum"]) -> "Sum":
        for metric in metrics:
            self.weighted_sum += metric.weighted_sum.to(self.device)
        return self
