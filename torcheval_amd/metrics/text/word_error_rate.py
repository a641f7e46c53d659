"""WordErrorRate class metric (parity: metrics/text/word_error_rate.py)."""

from typing import List, Optional, Union

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.text import (
    _word_error_rate_compute,
    _word_error_rate_update,
)
from torcheval_amd.metrics.text._sum_states import _SumStates

__all__ = ["WordErrorRate"]


class WordErrorRate(_SumStates):
    """Word error rate (native C++ edit distance)."""

    _names = ("errors", "total")

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("errors", torch.tensor(0, dtype=torch.float, device=self.device), merge="sum")
        self._add_state("total", torch.tensor(0, dtype=torch.float, device=self.device), merge="sum")

    @inference_update
    def update(self, input: Union[str, List[str]], target: Union[str, List[str]]) -> "WordErrorRate":
        errors, total = _word_error_rate_update(input, target)
        self.errors += errors.to(self.device)
        self.total += total.to(self.device)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _word_error_rate_compute(self.errors, self.total)
