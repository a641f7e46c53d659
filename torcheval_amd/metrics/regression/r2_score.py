"""R2Score class metric (parity: metrics/regression/r2_score.py)."""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.functional.regression import (
    _r2_score_compute,
    _r2_score_param_check,
    _r2_score_update,
    _r2_score_update_input_check,
)
from torcheval_amd.metrics.functional.regression._common import fused_regression_update
from torcheval_amd.ops import rowsums as _rs
from torcheval_amd.metrics._pending import PendingMixin, pending_states
from torcheval_amd.metrics.metric import Metric

__all__ = ["R2Score"]

# states folded from the K5 deferred-mode pending sums when read (metrics/_pending.py)
_PEND = ("sum_squared_obs", "sum_obs", "sum_squared_residual", "num_obs")


@pending_states(*_PEND)
class R2Score(PendingMixin, Metric[torch.Tensor]):
    """Coefficient of determination (optionally adjusted).  Functional version: ``r2_score``."""

    def __init__(
        self, *, multioutput: str = "uniform_average", num_regressors: int = 0, device: Optional[torch.device] = None
    ) -> None:
        super().__init__(device=device)
        _r2_score_param_check(multioutput, num_regressors)
        self.multioutput = multioutput
        self.num_regressors = num_regressors
        for name in ("sum_squared_obs", "sum_obs", "sum_squared_residual", "num_obs"):
            self._add_state(name, torch.tensor(0.0, device=self.device))

    def update(self, input: torch.Tensor, target: torch.Tensor) -> "R2Score":
        _r2_score_update_input_check(input, target)
        if fused_regression_update(
            self, input, target, None,
            [("sum_squared_obs", _rs.WTT), ("sum_obs", _rs.WT), ("sum_squared_residual", _rs.SSE)],
            [("num_obs", _rs.COUNT)],
        ):
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            sso, so, ssr, n = _r2_score_update(input, target)
            if self.sum_squared_obs.ndim == 0 and sso.ndim == 1:
                self.sum_squared_obs, self.sum_obs, self.sum_squared_residual = sso, so, ssr
            else:
                self.sum_squared_obs += sso
                self.sum_obs += so
                self.sum_squared_residual += ssr
            self.num_obs += n
            return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _r2_score_compute(
            self.sum_squared_obs, self.sum_obs, self.sum_squared_residual, self.num_obs,
            self.multioutput, self.num_regressors,
        )

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["R2Score"]) -> "R2Score":
        for metric in metrics:
            if self.sum_squared_obs.ndim == 0 and metric.sum_squared_obs.ndim == 1:
                self.sum_squared_obs = metric.sum_squared_obs.to(self.device)
                self.sum_obs = metric.sum_obs.to(self.device)
                self.sum_squared_residual = metric.sum_squared_residual.to(self.device)
            else:
                self.sum_squared_obs += metric.sum_squared_obs.to(self.device)
                self.sum_obs += metric.sum_obs.to(self.device)
                self.sum_squared_residual += metric.sum_squared_residual.to(self.device)
            self.num_obs += metric.num_obs.to(self.device)
        return self
