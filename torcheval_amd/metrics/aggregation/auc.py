"""AUC class metric (parity: metrics/aggregation/auc.py)."""

from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.functional.aggregation import (
    _auc_compute,
    _auc_update_input_check,
)
from torcheval_amd.metrics.metric import Metric, inference_update

__all__ = ["AUC"]


class AUC(Metric[torch.Tensor]):
    """Area under the curve of accumulated (x, y) points per task (trapezoid rule)."""

    def __init__(self, *, reorder: bool = True, n_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("x", [], merge="cat")
        self._add_state("y", [], merge="cat")
        self.n_tasks = n_tasks
        self.reorder = reorder

    @inference_update
    def update(self, x: torch.Tensor, y: torch.Tensor) -> "AUC":
        _auc_update_input_check(x, y, n_tasks=self.n_tasks)
        self.x.append(x.unsqueeze(0) if x.ndim == 1 else x)
        self.y.append(y.unsqueeze(0) if y.ndim == 1 else y)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if not self.x or not self.y:
            return torch.tensor([])
        return _auc_compute(torch.cat(self.x, dim=1), torch.cat(self.y, dim=1), reorder=self.reorder)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["AUC"]) -> "AUC":
        self._prepare_for_merge_state()
        for metric in metrics:
            if metric.x:
                self.x.append(torch.cat(metric.x, dim=1).to(self.device))
                self.y.append(torch.cat(metric.y, dim=1).to(self.device))
        return self

    @torch.inference_mode()
    def _prepare_for_merge_state(self) -> None:
        if self.x and self.y:
            self.x = [torch.cat(self.x, dim=1)]
            self.y = [torch.cat(self.y, dim=1)]
