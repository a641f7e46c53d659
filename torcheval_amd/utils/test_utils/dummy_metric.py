"""Minimal Tensor / List / Dict state metrics used by core and toolkit tests
(parity with torcheval/utils/test_utils/dummy_metric.py:19,48,80)."""

from collections import defaultdict
from typing import Iterable, Optional, TypeVar

import torch

from torcheval_amd.metrics.metric import Metric, _ZeroTensor

TDummy = TypeVar("TDummy")


class DummySumMetric(Metric[torch.Tensor]):
    """Sum of all update values; state declared ``merge="sum"`` (typed sync path)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("sum", torch.tensor(0.0, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, x: torch.Tensor) -> "DummySumMetric":
        self.sum += x
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return self.sum

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["DummySumMetric"]) -> "DummySumMetric":
        for metric in metrics:
            self.sum += metric.sum.to(self.device)
        return self


class DummySumListStateMetric(Metric[torch.Tensor]):
    """Keeps every update in a list state (untyped: exercises the merge_state sync path)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("x", [])

    @torch.inference_mode()
    def update(self, x: torch.Tensor) -> "DummySumListStateMetric":
        self.x.append(x.to(self.device))
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return sum(tensor.sum() for tensor in self.x)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["DummySumListStateMetric"]) -> "DummySumListStateMetric":
        for metric in metrics:
            self.x.extend(element.to(self.device) for element in metric.x)
        return self


class DummySumDictStateMetric(Metric[torch.Tensor]):
    """Dict state keyed by string (untyped)."""

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("x", defaultdict(_ZeroTensor(self.device)))

    @torch.inference_mode()
    def update(self, k: str, v: torch.Tensor) -> "DummySumDictStateMetric":
        self.x[k] += v
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return self.x

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["DummySumDictStateMetric"]) -> "DummySumDictStateMetric":
        for metric in metrics:
            for k in metric.x.keys():
                self.x[k] += metric.x[k].to(self.device)
        return self
