"""MeanSquaredError class metric (parity: metrics/regression/mean_squared_error.py)."""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.functional.regression import (
    _mean_squared_error_compute,
    _mean_squared_error_param_check,
    _mean_squared_error_update,
    _mean_squared_error_update_input_check,
)
from torcheval_amd.metrics.functional.regression._common import fused_regression_update
from torcheval_amd.ops import rowsums as _rs
from torcheval_amd.metrics._pending import PendingMixin, pending_states
from torcheval_amd.metrics.metric import Metric

__all__ = ["MeanSquaredError"]

# states folded from the K5 deferred-mode pending sums when read (metrics/_pending.py)
_PEND = ("sum_squared_error", "sum_weight")


@pending_states(*_PEND)
class MeanSquaredError(PendingMixin, Metric[torch.Tensor]):
    """Mean squared error; ``multioutput`` in uniform_average | raw_values.
    Functional version: ``mean_squared_error``."""

    def __init__(self, *, multioutput: str = "uniform_average", device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        _mean_squared_error_param_check(multioutput)
        self.multioutput = multioutput
        self._add_state("sum_squared_error", torch.tensor(0.0, device=self.device))
        self._add_state("sum_weight", torch.tensor(0.0, device=self.device))

    def update(
        self, input: torch.Tensor, target: torch.Tensor, *, sample_weight: Optional[torch.Tensor] = None
    ) -> "MeanSquaredError":
        _mean_squared_error_update_input_check(input, target, sample_weight)
        if fused_regression_update(self, input, target, sample_weight,
                                   [("sum_squared_error", _rs.WSSE)], [("sum_weight", _rs.W)]):
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            sse, sum_weight = _mean_squared_error_update(input, target, sample_weight)
            if self.sum_squared_error.ndim == 0 and sse.ndim == 1:
                self.sum_squared_error = sse
            else:
                self.sum_squared_error += sse
            self.sum_weight += sum_weight
            return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _mean_squared_error_compute(self.sum_squared_error, self.multioutput, self.sum_weight)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["MeanSquaredError"]) -> "MeanSquaredError":
        for metric in metrics:
            if self.sum_squared_error.ndim == 0 and metric.sum_squared_error.ndim == 1:
                self.sum_squared_error = metric.sum_squared_error.to(self.device)
            else:
                self.sum_squared_error += metric.sum_squared_error.to(self.device)
            self.sum_weight += metric.sum_weight.to(self.device)
        return self
