"""Mean class metric (parity: metrics/aggregation/mean.py)."""

import logging
from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.aggregation import _mean_update
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

_logger = logging.getLogger(__name__)

__all__ = ["Mean"]

_CODES = [_rs.code(_rs.WX, _rs.ADD), _rs.code(_rs.W, _rs.ADD)]


class Mean(Metric[torch.Tensor]):
    """Weighted mean of all inputs (float64 accumulators)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("weighted_sum", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")
        self._add_state("weights", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")

    def update(self, input: torch.Tensor, *, weight: Union[float, int, torch.Tensor] = 1.0) -> "Mean":
        if _rs.fast_ok(input, weight, self.weighted_sum, self.weights):
            # K5b: sum(w x) and sum(w) merged into both states in one launch (host twin on CPU);
            # the native op records no autograd, so no inference-mode guard is needed here
            tw = isinstance(weight, torch.Tensor)
            _rs.update(input, None, weight if tw else None, 1.0 if tw else float(weight),
                       [self.weighted_sum, self.weights], _CODES)
            return self
        return self._update_aten(input, weight)

    @torch.inference_mode()
    def _update_aten(self, input: torch.Tensor, weight) -> "Mean":
        weighted_sum, weights = _mean_update(input, weight)
        self.weighted_sum += weighted_sum
        self.weights += weights
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if not self.weighted_sum:
            _logger.warning("No calls to update() have been made - returning 0.0")
            return torch.tensor(0.0, dtype=torch.float64)
        return self.weighted_sum / self.weights

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Mean"]) -> "Mean":
        for metric in metrics:
            self.weighted_sum += metric.weighted_sum.to(self.device)
            self.weights += metric.weights.to(self.device)
        return self

