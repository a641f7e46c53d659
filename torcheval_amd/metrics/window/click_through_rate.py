"""Windowed click-through rate (parity: metrics/window/click_through_rate.py:19)."""

from typing import Optional, Tuple, Union

import torch

from torcheval_amd.metrics.functional.ranking import (
    _click_through_rate_compute,
    _click_through_rate_input_check,
    _click_through_rate_update,
)
from torcheval_amd.metrics.window._ring import _WindowedSums
from torcheval_amd.ops import rowsums as _rs


class WindowedClickThroughRate(_WindowedSums):
    """CTR over the last ``max_num_updates`` updates (and lifetime when ``enable_lifetime``).

    ``compute()`` returns ``(lifetime, windowed)`` or ``windowed``; empty tensors before any update."""

    _WINDOW = (("windowed_click_total", torch.float64), ("windowed_weight_total", torch.float64))
    _LIFETIME = (("click_total", torch.float64), ("weight_total", torch.float64))

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
            enable_lifetime=enable_lifetime, device=device,
        )

    def update(self, input: torch.Tensor, weights: Union[torch.Tensor, float, int] = 1.0):
        slot_c, slot_w = self._slot_views()
        if _rs.weight_ok(input, weights) and _rs.supported(
            input, weights if isinstance(weights, torch.Tensor) else None, states=(slot_c, slot_w)
        ):
            # K5b: the ring-slot write and the lifetime accumulation in one launch
            _click_through_rate_input_check(input, weights, num_tasks=self.num_tasks)
            outs = [(slot_c, _rs.WX, _rs.SET), (slot_w, _rs.W, _rs.SET)]
            if self.enable_lifetime:
                outs += [(self.click_total, _rs.WX, _rs.ADD), (self.weight_total, _rs.W, _rs.ADD)]
            _rs.update_states(input, None, weights, outs, rows=self.num_tasks)
            self._advance()
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            click_total, weight_total = _click_through_rate_update(input, weights, num_tasks=self.num_tasks)
            if self.enable_lifetime:
                self.click_total += click_total
                self.weight_total += weight_total
            self._push((click_total, weight_total))
            return self

    @torch.inference_mode()
    def compute(self) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        if self.total_updates == 0:
            return self._empty_result()
        click, weight = self._window_totals()
        windowed = _click_through_rate_compute(click, weight)
        if self.enable_lifetime:
            return _click_through_rate_compute(self.click_total, self.weight_total), windowed
        return windowed
