"""Throughput class metric (parity: metrics/aggregation/throughput.py)."""

import logging
from typing import Iterable, Optional

import torch

from torcheval_amd.metrics.metric import Metric, inference_update

_logger = logging.getLogger(__name__)

__all__ = ["Throughput"]


class Throughput(Metric[float]):
    """Items processed per second; merged across ranks as (sum of items) / (max elapsed)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("num_total", 0.0)
        self._add_state("elapsed_time_sec", 0.0)

    @inference_update
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
