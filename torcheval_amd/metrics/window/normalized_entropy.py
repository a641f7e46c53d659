"""Windowed binary normalized entropy (parity: metrics/window/normalized_entropy.py:19).

On the GPU each update is one K6 launch; the probability-range check is a device flag that
``compute()`` raises on (as ``BinaryNormalizedEntropy``)."""

from typing import Optional, Tuple, Union

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.classification.binary_normalized_entropy import (
    _baseline_update,
    _binary_normalized_entropy_update,
    _ne_device_error,
)
from torcheval_amd.metrics.window._ring import _WindowedSums


class WindowedBinaryNormalizedEntropy(_WindowedSums):
    """Normalized BCE over the last ``max_num_updates`` updates (+ lifetime) per task."""

    _err_merge = "first"  # int32[6] record: flag + packed 64-bit range keys

    _WINDOW = (
        ("windowed_total_entropy", torch.float64),
        ("windowed_num_examples", torch.float64),
        ("windowed_num_positive", torch.float64),
    )
    _LIFETIME = (
        ("total_entropy", torch.float64),
        ("num_examples", torch.float64),
        ("num_positive", torch.float64),
    )

    def __init__(
        self,
        *,
        from_logits: bool = False,
        num_tasks: int = 1,
        max_num_updates: int = 100,
        enable_lifetime: bool = True,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(
            num_tasks=num_tasks, max_num_updates=max_num_updates,
            enable_lifetime=enable_lifetime, device=device,
        )
        self.from_logits = from_logits
        self._err: Optional[torch.Tensor] = None

    @inference_update
    def update(
        self, input: torch.Tensor, target: torch.Tensor, *, weight: Optional[torch.Tensor] = None
    ):
        if input.is_cuda and self._err is None:
            self._err = torch.zeros(6, dtype=torch.int32, device=input.device)
        self._x_dtype = input.dtype
        ce, pos, ex = _binary_normalized_entropy_update(
            input, target, self.from_logits, self.num_tasks, weight,
            err=self._err if input.is_cuda else None,
        )
        if self.enable_lifetime:
            self.total_entropy += ce
            self.num_examples += ex
            self.num_positive += pos
        self._push((ce, ex, pos))
        return self

    def _check_device_errors(self) -> None:
        if self._err is not None:
            _ne_device_error(self._err, self.from_logits, getattr(self, "_x_dtype", torch.float32))

    @torch.inference_mode()
    def compute(self) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        self._check_device_errors()
        if self.total_updates == 0:
            return self._empty_result()
        ce, ex, pos = self._window_totals()
        windowed = (ce / ex) / _baseline_update(pos, ex)
        if self.enable_lifetime:
            lifetime = (self.total_entropy / self.num_examples) / _baseline_update(
                self.num_positive, self.num_examples
            )
            return lifetime, windowed
        return windowed
