"""Windowed weighted calibration (parity: metrics/window/weighted_calibration.py:19)."""

from typing import Optional, Tuple, Union

import torch

from torcheval_amd.metrics.functional.ranking import _weighted_calibration_update
from torcheval_amd.metrics.functional.ranking._rank_common import _num_tasks_check
from torcheval_amd.metrics.window._ring import _WindowedSums
from torcheval_amd.ops import rowsums as _rs

_EPS64 = torch.finfo(torch.float64).eps


class WindowedWeightedCalibration(_WindowedSums):
    """sum(w * input) / sum(w * target) over the last ``max_num_updates`` updates (+ lifetime)."""

    _WINDOW = (
        ("windowed_weighted_input_sum", torch.float64),
        ("windowed_weighted_target_sum", torch.float64),
    )
    _LIFETIME = (("weighted_input_sum", torch.float64), ("weighted_target_sum", torch.float64))

    def __init__(
        self,
        *,
        num_tasks: int = 1,
        max_num_updates: int = 100,
        enable_lifetime: bool = True,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(
            num_tasks=num_tasks, max_num_updates=max_num_updates,
            enable_lifetime=enable_lifetime, device=device, check_max=False,
        )

    def update(
        self, input: torch.Tensor, target: torch.Tensor, weight: Union[float, int, torch.Tensor] = 1.0
    ):
        slot_i, slot_t = self._slot_views()
        if input.shape == target.shape and _rs.weight_ok(input, weight) and _rs.supported(
            input, target, weight if isinstance(weight, torch.Tensor) else None, states=(slot_i, slot_t)
        ):
            _num_tasks_check(input, self.num_tasks)
            outs = [(slot_i, _rs.WX, _rs.SET), (slot_t, _rs.WT, _rs.SET)]
            if self.enable_lifetime:
                outs += [(self.weighted_input_sum, _rs.WX, _rs.ADD), (self.weighted_target_sum, _rs.WT, _rs.ADD)]
            _rs.update_states(input, target, weight, outs, rows=self.num_tasks)
            self._advance()
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            wi, wt = _weighted_calibration_update(input, target, weight, num_tasks=self.num_tasks)
            if self.enable_lifetime:
                self.weighted_input_sum += wi
                self.weighted_target_sum += wt
            self._push((wi, wt))
            return self

    @torch.inference_mode()
    def compute(self) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        if self.total_updates == 0:
            return self._empty_result()
        wi, wt = self._window_totals()
        windowed = wi / torch.clamp(wt, min=_EPS64)
        if self.enable_lifetime:
            lifetime = self.weighted_input_sum / torch.clamp(self.weighted_target_sum, min=_EPS64)
            return lifetime, windowed
        return windowed
