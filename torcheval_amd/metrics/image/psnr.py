"""PSNR, class API (parity: metrics/image/psnr.py:24-129).

``data_range`` is recomputed from the merged target min / max when auto-ranging, so the
states use the metric's own ``merge_state`` during sync (merge kind ``None``).

ROCm batches longer than 32K elements run K5b in deferred mode (metrics/_pending.py): the launch
adds each block's FP64 SSE / count and its target min / max to pending slots and ends with its
last load; the states fold them (sums added, extrema merged, data_range set) when next read.
Shorter batches, CPU tensors and torch.compile merge in-launch as before.
"""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.functional.image import (
    _psnr_compute,
    _psnr_input_check,
    _psnr_param_check,
    _psnr_update,
)
from torcheval_amd.metrics._pending import PendingMixin, RowSumsSpec, pending_states
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import compiling
from torcheval_amd.ops import rowsums as _rs

_NAMES = ("sum_squared_error", "num_observations", "min_target", "max_target", "data_range")
_FIXED = ((_rs.SSE, _rs.ADD), (_rs.COUNT, _rs.ADD))
_AUTO = _FIXED + ((_rs.TMIN, _rs.MIN), (_rs.TMAX, _rs.MAX), (_rs.RANGE, _rs.SET))
_SPECS = {False: RowSumsSpec(_NAMES[:2], tuple(_rs.code(s, o) for s, o in _FIXED), 1),
          True: RowSumsSpec(_NAMES, tuple(_rs.code(s, o) for s, o in _AUTO), 1)}


@pending_states(*_NAMES)
class PeakSignalNoiseRatio(PendingMixin, Metric[torch.Tensor]):
    """Peak signal-to-noise ratio over all updates; ``data_range=None`` tracks the target range."""

    def __init__(self, data_range: Optional[float] = None, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        _psnr_param_check(data_range=data_range)
        self.auto_range = data_range is None
        self._add_state("data_range", torch.tensor(0.0 if data_range is None else data_range, device=self.device))
        self._add_state("num_observations", torch.tensor(0.0, device=self.device))
        self._add_state("sum_squared_error", torch.tensor(0.0, device=self.device))
        self._add_state("min_target", torch.tensor(torch.inf, device=self.device))
        self._add_state("max_target", torch.tensor(-torch.inf, device=self.device))

    def update(self, input: torch.Tensor, target: torch.Tensor) -> "PeakSignalNoiseRatio":
        _psnr_input_check(input, target)
        states = tuple(self._raw_state(n) for n in _NAMES)  # no fold: an update only adds
        if self._fusable(input, target, states) and _rs.supported(input, target, states=states):
            spec = _SPECS[self.auto_range]
            if self._rowsums_deferred(input, None, 1.0, spec, t=target):
                return self
            # K5b: SSE, count and (auto range) target min / max / range merged in one launch
            codes = _AUTO if self.auto_range else _FIXED
            _rs.update_states(input, target, None, [(st, s, o) for st, (s, o) in zip(states, codes)])
            return self
        with torch.inference_mode():  # the ATen path (the native op records no autograd)
            sse, n = _psnr_update(input, target)
            self.sum_squared_error = self.sum_squared_error + sse
            self.num_observations = self.num_observations + n
            if self.auto_range:
                self.min_target = torch.minimum(target.min(), self.min_target)
                self.max_target = torch.maximum(target.max(), self.max_target)
                self.data_range = self.max_target - self.min_target
            return self

    def _fusable(self, input: torch.Tensor, target: torch.Tensor, states) -> bool:
        """In-place accumulation keeps the reference's out-of-place dtype promotion only when
        no state would be promoted (and bool inputs keep the ATen error)."""
        if input.dtype == torch.bool or target.dtype == torch.bool or compiling():
            return False  # (torch.compile: the ATen form, traceable end to end)
        sse, _, tmin, tmax, rng = states
        diff = torch.result_type(input, target)
        pt = torch.promote_types
        return (pt(sse.dtype, diff) == sse.dtype
                and (not self.auto_range or (pt(tmin.dtype, target.dtype) == tmin.dtype
                                             and pt(tmax.dtype, target.dtype) == tmax.dtype
                                             and rng.dtype == tmax.dtype)))

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _psnr_compute(self.sum_squared_error, self.num_observations, self.data_range)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["PeakSignalNoiseRatio"]) -> "PeakSignalNoiseRatio":
        for metric in metrics:
            self.num_observations = self.num_observations + metric.num_observations.to(self.device)
            self.sum_squared_error = self.sum_squared_error + metric.sum_squared_error.to(self.device)
            if self.auto_range:
                self.min_target = torch.minimum(self.min_target, metric.min_target.to(self.device))
                self.max_target = torch.maximum(self.max_target, metric.max_target.to(self.device))
        if self.auto_range:
            self.data_range = self.max_target - self.min_target
        return self
