"""Aggregation metrics, class API (parity: metrics/aggregation/*.py).

``Sum``/``Mean`` states are ``merge="sum"``, ``Max``/``Min`` ``merge="max"/"min"`` (one RCCL
all-reduce each), ``Cat``/``AUC`` lists ``merge="cat"`` (all-gather-v).  ``Throughput`` keeps
Python-number states with a custom merge (elapsed time is a MAX across ranks).
"""

import logging
from typing import Iterable, Optional, TypeVar, Union

import torch

from torcheval_amd.metrics.functional.aggregation import (
    _auc_compute,
    _auc_update_input_check,
    _mean_update,
    _sum_update,
)
from torcheval_amd.metrics.metric import Metric

__all__ = ["AUC", "Cat", "Max", "Mean", "Min", "Sum", "Throughput"]
__doc_name__ = "Aggregation Metrics"

_logger = logging.getLogger(__name__)
TSelf = TypeVar("TSelf")


class AUC(Metric[torch.Tensor]):
    """Area under the curve of accumulated (x, y) points per task (trapezoid rule)."""

    def __init__(self, *, reorder: bool = True, n_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("x", [], merge="cat")
        self._add_state("y", [], merge="cat")
        self.n_tasks = n_tasks
        self.reorder = reorder

    @torch.inference_mode()
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


class Cat(Metric[torch.Tensor]):
    """Concatenation of all updates along ``dim``."""

    def __init__(self, *, dim: int = 0, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("dim", dim)
        self._add_state("inputs", [])

    @torch.inference_mode()
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


class Max(Metric[torch.Tensor]):
    """Running maximum of all inputs."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("max", torch.tensor(float("-inf"), device=self.device), merge="max")

    @torch.inference_mode()
    def update(self, input: torch.Tensor) -> "Max":
        self.max = torch.max(self.max, torch.max(input))
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return self.max

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Max"]) -> "Max":
        for metric in metrics:
            self.max = torch.max(self.max, metric.max.to(self.device))
        return self


class Min(Metric[torch.Tensor]):
    """Running minimum of all inputs."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("min", torch.tensor(float("inf"), device=self.device), merge="min")

    @torch.inference_mode()
    def update(self, input: torch.Tensor) -> "Min":
        self.min = torch.min(self.min, torch.min(input))
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return self.min

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Min"]) -> "Min":
        for metric in metrics:
            self.min = torch.min(self.min, metric.min.to(self.device))
        return self


class Mean(Metric[torch.Tensor]):
    """Weighted mean of all inputs (float64 accumulators)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("weighted_sum", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")
        self._add_state("weights", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")

    @torch.inference_mode()
    def update(self, input: torch.Tensor, *, weight: Union[float, int, torch.Tensor] = 1.0) -> "Mean":
        weighted_sum, weights = _mean_update(input, weight)
        self.weighted_sum += weighted_sum
        self.weights += weights
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if not self.weighted_sum:
            _logger.warning("No calls to update() have been made - returning 0.0")
            return torch.tensor(0.0, dtype=torch.float64)
        return self.weighted_sum / self.weights

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Mean"]) -> "Mean":
        for metric in metrics:
            self.weighted_sum += metric.weighted_sum.to(self.device)
            self.weights += metric.weights.to(self.device)
        return self


class Sum(Metric[torch.Tensor]):
    """Weighted sum of all inputs (float64 accumulator)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("weighted_sum", torch.tensor(0.0, device=self.device, dtype=torch.float64), merge="sum")

    @torch.inference_mode()
    def update(self, input: torch.Tensor, *, weight: Union[float, int, torch.Tensor] = 1.0) -> "Sum":
        self.weighted_sum += _sum_update(input, weight)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return self.weighted_sum

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Sum"]) -> "Sum":
        for metric in metrics:
            self.weighted_sum += metric.weighted_sum.to(self.device)
        return self


class Throughput(Metric[float]):
    """Items processed per second; merged across ranks as (sum of items) / (max elapsed)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("num_total", 0.0)
        self._add_state("elapsed_time_sec", 0.0)

    @torch.inference_mode()
    def update(self, num_processed: int, elapsed_time_sec: float) -> "Throughput":
        if num_processed < 0:
            raise ValueError(
                f"Expected num_processed to be a non-negative number, but received {num_processed}."
            )
        if elapsed_time_sec <= 0:
            raise ValueError(
                f"Expected elapsed_time_sec to be a positive number, but received {elapsed_time_sec}."
            )
        self.elapsed_time_sec += elapsed_time_sec
        self.num_total += num_processed
        return self

    @torch.inference_mode()
    def compute(self) -> float:
        if not self.elapsed_time_sec:
            _logger.warning("No calls to update() have been made - returning 0.0")
            return 0.0
        return self.num_total / self.elapsed_time_sec

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["Throughput"]) -> "Throughput":
        for metric in metrics:
            self.num_total += metric.num_total
            self.elapsed_time_sec = max(self.elapsed_time_sec, metric.elapsed_time_sec)
        return self
