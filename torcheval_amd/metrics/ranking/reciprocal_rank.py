"""ReciprocalRank class metric (parity: metrics/ranking/reciprocal_rank.py)."""

import torch

from torcheval_amd.metrics.metric import inference_update

from torcheval_amd.metrics.functional.ranking.reciprocal_rank import _reciprocal_rank
from torcheval_amd.metrics.ranking._score_list import _RankScoreList

__all__ = ["ReciprocalRank"]


class ReciprocalRank(_RankScoreList):
    """Per-sample reciprocal rank scores, concatenated over updates."""

    @inference_update
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "ReciprocalRank":
        self.scores.append(_reciprocal_rank(input, target, self.k, self._err_for(input)))
        return self
