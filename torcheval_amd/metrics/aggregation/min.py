"""Min class metric (parity: metrics/aggregation/min.py)."""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.metric import Metric, inference_update

__all__ = ["Min"]


class Min(Metric[torch.Tensor]):
    """Running minimum of all inputs."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("min", torch.tensor(float("inf"), device=self.device), merge="min")

    @inference_update
    def update(self, input: torch.Tensor) -> "Min":
        self.min = torch.min(self.min, torch.min(input))
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return self.min if self._tea_sb is None else self.min.clone()  # buffer reset is in place

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Min"]) -> "Min":
        for metric in metrics:
            self.min = torch.min(self.min, metric.min.to(self.device))
        return self
