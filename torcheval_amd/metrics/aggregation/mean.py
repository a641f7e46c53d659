"""Mean class metric (parity: metrics/aggregation/mean.py)."""

import logging
from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.aggregation import _mean_update
from torcheval_amd.metrics._pending import PendingMixin, RowSumsSpec, pending_states
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

_logger = logging.getLogger(__name__)

__all__ = ["Mean"]

_CODES = [_rs.code(_rs.WX, _rs.ADD), _rs.code(_rs.W, _rs.ADD)]


# long ROCm batches add to device pending sums, folded into the states when they are read
_SPEC = RowSumsSpec(("weighted_sum", "weights"), tuple(_CODES), 1)


@pending_states("weighted_sum", "weights")
class Mean(PendingMixin, Metric[torch.Tensor]):
    """Weighted mean of all inputs (float64 accumulators)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("weighted_sum", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")
        self._add_state("weights", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")

    def update(self, input: torch.Tensor, *, weight: Union[float, int, torch.Tensor] = 1.0) -> "Mean":
        d = self.__dict__
        ws, wt = d["_pv_weighted_sum"], d["_pv_weights"]  # no fold: an update only adds
        if _rs.fast_ok(input, weight, ws, wt):
            # K5b: sum(w x) and sum(w) merged into both states in one launch (host twin on CPU);
            # the native op records no autograd, so no inference-mode guard is needed here
            tw = isinstance(weight, torch.Tensor)
            w, wsc = (weight, 1.0) if tw else (None, float(weight))
            if not self._rowsums_deferred(input, w, wsc, _SPEC):
                _rs.update(input, None, w, wsc, [ws, wt], _CODES)
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

