"""Shared base of the text class metrics whose states are additive sums."""

from typing import Iterable

import torch

from torcheval_amd.metrics.metric import Metric


class _SumStates(Metric[torch.Tensor]):
    _names: tuple = ()

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["_SumStates"]):
        for metric in metrics:
            for n in self._names:
                getattr(self, n).add_(getattr(metric, n).to(self.device))
        return self
