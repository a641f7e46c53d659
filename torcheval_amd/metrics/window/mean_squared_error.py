"""Windowed mean squared error (parity: metrics/window/mean_squared_error.py:23).

Each update is one K5 column-moments launch on the GPU (see ``functional.regression``)."""

from typing import Optional, Tuple, Union

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.regression import (
    _mean_squared_error_compute,
    _mean_squared_error_param_check,
    _mean_squared_error_update,
)
from torcheval_amd.metrics.window._ring import _WindowedSums


class WindowedMeanSquaredError(_WindowedSums):
    """MSE over the last ``max_num_updates`` updates (+ lifetime); ``num_tasks`` = output columns."""

    _WINDOW = (("windowed_sum_squared_error", torch.float32), ("windowed_sum_weight", torch.float32))
    _LIFETIME = (("sum_squared_error", torch.float32), ("sum_weight", torch.float32))

    def __init__(
        self,
        *,
        num_tasks: int = 1,
        max_num_updates: int = 100,
        enable_lifetime: bool = True,
        multioutput: str = "uniform_average",
        device: Optional[torch.device] = None,
    ) -> None:
        _mean_squared_error_param_check(multioutput)
        super().__init__(
            num_tasks=num_tasks, max_num_updates=max_num_updates,
            enable_lifetime=enable_lifetime, device=device, lifetime_shape=(),
        )
        self.multioutput = multioutput

    @inference_update
    def update(
        self, input: torch.Tensor, target: torch.Tensor, *, sample_weight: Optional[torch.Tensor] = None
    ):
        sse, sw = _mean_squared_error_update(input, target, sample_weight)
        self._window_mean_squared_error_update_input_check(input, target, sample_weight, self.num_tasks)
        if self.enable_lifetime:
            if self.sum_squared_error.ndim == 0 and sse.ndim == 1:
                self.sum_squared_error = sse.to(torch.float32).clone()
            else:
                self.sum_squared_error += sse
            self.sum_weight += sw
        self._push((sse, sw))
        return self

    def _merge_lifetime(self, metric: "WindowedMeanSquaredError") -> None:
        other = metric.sum_squared_error.to(self.device)
        if self.sum_squared_error.ndim == 0 and other.ndim == 1:
            self.sum_squared_error = other.clone()
        else:
            self.sum_squared_error = self.sum_squared_error + other
        self.sum_weight = self.sum_weight + metric.sum_weight.to(self.device)

    @torch.inference_mode()
    def compute(self) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        if self.total_updates == 0:
            return self._empty_result()
        sse, sw = self._window_totals()
        windowed = _mean_squared_error_compute(sse, self.multioutput, sw)
        if self.enable_lifetime:
            lifetime = _mean_squared_error_compute(self.sum_squared_error, self.multioutput, self.sum_weight)
            return lifetime.squeeze(), windowed.squeeze()
        return windowed.squeeze()

    def _window_mean_squared_error_update_input_check(
        self, input: torch.Tensor, target: torch.Tensor, sample_weight: Optional[torch.Tensor],
        num_tasks: int = 1,
    ) -> None:
        if num_tasks == 1:
            if len(input.shape) > 1:
                raise ValueError(
                    f"`num_tasks = 1`, `input` is expected to be one-dimensional tensor, but got shape ({input.shape})."
                )
        elif len(input.shape) == 1 or input.shape[1] != num_tasks:
            raise ValueError(
                f"`num_tasks = {num_tasks}`, `input`'s shape is expected to be (num_samples, {num_tasks}), but got shape ({input.shape})."
            )
