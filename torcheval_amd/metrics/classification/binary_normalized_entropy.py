"""Binary normalized entropy, class API (parity: classification/binary_normalized_entropy.py:22).

GPU update = one K6 launch accumulating float64 (entropy, positives, examples) per task;
the probability-range check is a device flag raised at ``compute()`` (no per-update sync).
"""

from typing import Iterable, Optional, TypeVar

import torch

from torcheval_amd.metrics.functional.classification.binary_normalized_entropy import (
    _baseline_update,
    _binary_normalized_entropy_update,
    _ne_device_error,
)
from torcheval_amd.metrics.metric import Metric, inference_update

TNormalizedEntropy = TypeVar("TNormalizedEntropy")


class BinaryNormalizedEntropy(Metric[torch.Tensor]):
    """
    Normalized binary cross entropy per task (float64).

    Args:
        from_logits: ``input`` holds logits (BCE-with-logits) instead of probabilities.
        num_tasks: number of independent tasks (rows of a ``[num_tasks, n]`` input).
    Functional version: ``binary_normalized_entropy``.
    """

    _err_merge = "first"  # int32[6] record: flag + packed 64-bit range keys

    def __init__(
        self: TNormalizedEntropy,
        *,
        from_logits: bool = False,
        num_tasks: int = 1,
        device: Optional[torch.device] = None,
    ) -> None:
        super().__init__(device=device)
        self.from_logits = from_logits
        if num_tasks < 1:
            raise ValueError(
                "`num_tasks` value should be greater than and equal to 1, but received {num_tasks}. "
            )
        self.num_tasks = num_tasks
        self._err: Optional[torch.Tensor] = None
        for name in ("total_entropy", "num_examples", "num_positive"):
            self._add_state(
                name, torch.zeros(num_tasks, dtype=torch.float64, device=self.device), merge="sum"
            )

    @inference_update
    def update(
        self: TNormalizedEntropy,
        input: torch.Tensor,
        target: torch.Tensor,
        *,
        weight: Optional[torch.Tensor] = None,
    ) -> TNormalizedEntropy:
        input = input.to(self.device)
        target = target.to(self.device)
        if weight is not None:
            weight = weight.to(self.device)
        if input.is_cuda and self._err is None:
            self._err = torch.zeros(6, dtype=torch.int32, device=input.device)
        self._x_dtype = input.dtype
        cross_entropy, num_positive, num_examples = _binary_normalized_entropy_update(
            input, target, self.from_logits, self.num_tasks, weight,
            err=self._err if input.is_cuda else None,
        )
        self.total_entropy += cross_entropy
        self.num_examples += num_examples
        self.num_positive += num_positive
        return self

    def _check_device_errors(self) -> None:
        if self._err is not None:
            _ne_device_error(self._err, self.from_logits, getattr(self, "_x_dtype", torch.float32))

    @torch.inference_mode()
    def compute(self: TNormalizedEntropy) -> torch.Tensor:
        """Normalized entropy per task; empty tensor if some task has no examples."""
        self._check_device_errors()
        if torch.any(self.num_examples == 0.0):
            return torch.empty(0)
        baseline_entropy = _baseline_update(self.num_positive, self.num_examples)
        cross_entropy = self.total_entropy / self.num_examples
        return cross_entropy / baseline_entropy

    @torch.inference_mode()
    def merge_state(self: TNormalizedEntropy, metrics: Iterable[TNormalizedEntropy]) -> TNormalizedEntropy:
        for metric in metrics:
            self.total_entropy += metric.total_entropy.to(self.device)
            self.num_examples += metric.num_examples.to(self.device)
            self.num_positive += metric.num_positive.to(self.device)
        return self
