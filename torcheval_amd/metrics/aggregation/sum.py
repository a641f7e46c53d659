"""Sum class metric (parity: metrics/aggregation/sum.py)."""

from typing import Iterable, Optional, Union

import torch

from torcheval_amd.metrics.functional.aggregation import _sum_update
from torcheval_amd.metrics._pending import PendingMixin, RowSumsSpec, pending_states
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.ops import rowsums as _rs

__all__ = ["Sum"]

_CODES = [_rs.code(_rs.WX, _rs.ADD)]
# long ROCm batches add to device pending sums, folded into the state when it is read
_SPEC = RowSumsSpec(("weighted_sum",), tuple(_CODES), 1)


@pending_states("weighted_sum")
class Sum(PendingMixin, Metric[torch.Tensor]):
    """Weighted sum of all inputs (float64 accumulator)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("weighted_sum", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")

    def update(self, input: torch.Tensor, *, weight: Union[float, int, torch.Tensor] = 1.0) -> "Sum":
        ws = self.__dict__["_pv_weighted_sum"]  # no fold: an update only adds
        if _rs.fast_ok(input, weight, ws):  # K5b, one launch (host twin on CPU)
            tw = isinstance(weight, torch.Tensor)
            wt, wsc = (weight, 1.0) if tw else (None, float(weight))
            if not self._rowsums_deferred(input, wt, wsc, _SPEC):
                _rs.update(input, None, wt, wsc, [ws], _CODES)
            return self
        return self._update_aten(input, weight)

    @torch.inference_mode()
    def _update_aten(self, input: torch.Tensor, weight) -> "Sum":
        self.weighted_sum += _sum_update(input, weight)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        # a copy once the state lives in a state buffer: reset() then restores it in place
        return self.weighted_sum if self._tea_sb is None else self.weighted_sum.clone()

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Sum"]) -> "Sum":
        for metric in metrics:
            self.weighted_sum += metric.weighted_sum.to(self.device)
        return self
