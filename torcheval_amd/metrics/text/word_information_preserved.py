"""WordInformationPreserved class metric (parity: metrics/text/word_information_preserved.py)."""

from typing import List, Optional, Union

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.text import (
    _word_information_preserved_compute,
    _word_information_preserved_update,
)
from torcheval_amd.metrics.text._sum_states import _SumStates

__all__ = ["WordInformationPreserved"]


class WordInformationPreserved(_SumStates):
    """Word information preserved (native C++ edit distance)."""

    _names = ("correct_total", "input_total", "target_total")

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        for n in self._names:
            self._add_state(n, torch.tensor(0, dtype=torch.float64, device=self.device), merge="sum")

    @inference_update
    def update(self, input: Union[str, List[str]], target: Union[str, List[str]]) -> "WordInformationPreserved":
        c, t, i = _word_information_preserved_update(input, target)
        self.correct_total += c.to(self.device)
        self.target_total += t.to(self.device)
        self.input_total += i.to(self.device)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _word_information_preserved_compute(self.correct_total, self.target_total, self.input_total)
