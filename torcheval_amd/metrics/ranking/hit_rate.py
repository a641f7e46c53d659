"""HitRate class metric (parity: metrics/ranking/hit_rate.py)."""

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.ranking.hit_rate import _hit_rate
from torcheval_amd.metrics.ranking._score_list import _RankScoreList

__all__ = ["HitRate"]


class HitRate(_RankScoreList):
    """Per-sample hit (target within top-k) scores, concatenated over updates."""

    @inference_update
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "HitRate":
        self.scores.append(_hit_rate(input, target, self.k, self._err_for(input)))
        return self
