"""Cat class metric (parity: metrics/aggregation/cat.py)."""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.metric import Metric, inference_update

__all__ = ["Cat"]


class Cat(Metric[torch.Tensor]):
    """Concatenation of all updates along ``dim``."""

    def __init__(self, *, dim: int = 0, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("dim", dim)
        self._add_state("inputs", [])

    @inference_update
    def update(self, input: torch.Tensor) -> "Cat":
        self.inputs.append(input)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if not self.inputs:
            return torch.empty(0)
        return torch.cat(self.inputs, dim=self.dim)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Cat"]) -> "Cat":
        for metric in metrics:
            if metric.inputs:
                self.inputs.append(torch.cat(metric.inputs, dim=metric.dim).to(self.device))
        return self

    @torch.inference_mode()
    def _prepare_for_merge_state(self) -> None:
        if self.inputs:
            self.inputs = [torch.cat(self.inputs, dim=self.dim)]
