"""Regression metrics, class API (parity: metrics/regression/{mean_squared_error,r2_score}.py).

States follow the reference, including the lazy promotion of the scalar states to per-output
vectors on the first 2-D update / merge.  Because state shapes can differ across ranks they
use the metric's own ``merge_state`` during distributed sync (merge kind ``None``).
"""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.functional.regression import (
    _mean_squared_error_compute,
    _mean_squared_error_param_check,
    _mean_squared_error_update,
    _r2_score_compute,
    _r2_score_param_check,
    _r2_score_update,
)
from torcheval_amd.metrics.metric import Metric

__all__ = ["MeanSquaredError", "R2Score"]
__doc_name__ = "Regression Metrics"


class MeanSquaredError(Metric[torch.Tensor]):
    """Mean squared error; ``multioutput`` in uniform_average | raw_values.
    Functional version: ``mean_squared_error``."""

    def __init__(self, *, multioutput: str = "uniform_average", device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        _mean_squared_error_param_check(multioutput)
        self.multioutput = multioutput
        self._add_state("sum_squared_error", torch.tensor(0.0, device=self.device))
        self._add_state("sum_weight", torch.tensor(0.0, device=self.device))

    @torch.inference_mode()
    def update(
        self, input: torch.Tensor, target: torch.Tensor, *, sample_weight: Optional[torch.Tensor] = None
    ) -> "MeanSquaredError":
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


class R2Score(Metric[torch.Tensor]):
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

    @torch.inference_mode()
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "R2Score":
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
