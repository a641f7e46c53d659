"""Perplexity class metric (parity: metrics/text/perplexity.py)."""

from typing import Optional

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.text import _perplexity_compute, _perplexity_update
from torcheval_amd.metrics.text._sum_states import _SumStates
from torcheval_amd.ops.hostread import read_int

__all__ = ["Perplexity"]


class Perplexity(_SumStates):
    """Perplexity of token logits (fused K7 kernel on ROCm; label check deferred to compute)."""

    _names = ("sum_log_probs", "num_total")
    _err_words = 1  # K7 device flag: one int32 code

    def __init__(self, ignore_index: Optional[int] = None, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self.ignore_index = ignore_index
        self._err: Optional[torch.Tensor] = None
        self._add_state("sum_log_probs", torch.tensor(0.0, dtype=torch.float64, device=self.device), merge="sum")
        self._add_state("num_total", torch.tensor(0.0, dtype=torch.float64, device=self.device), merge="sum")

    @inference_update
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "Perplexity":
        if input.is_cuda and self._err is None:
            self._err = torch.zeros(1, dtype=torch.int32, device=input.device)
        s, n = _perplexity_update(input, target, self.ignore_index, err=self._err if input.is_cuda else None)
        self.sum_log_probs += s
        self.num_total += n
        return self

    def _check_device_errors(self) -> None:
        if self._err is not None and read_int(self._err) != 0:
            self._err.zero_()
            raise ValueError(
                "Class labels in `target` tensor cannot be larger than vocab_size minus one "
                "(detected on device in an earlier update())."
            )

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        self._check_device_errors()
        if self.num_total == 0.0:
            return torch.empty(0)
        return _perplexity_compute(self.sum_log_probs, self.num_total)
