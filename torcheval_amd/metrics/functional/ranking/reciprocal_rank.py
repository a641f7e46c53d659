"""Reciprocal rank, functional API (parity: functional/ranking/reciprocal_rank.py)."""

from typing import Optional

import torch

from torcheval_amd.metrics.functional.ranking._rank_common import _native_rank_scores, _rank_input_check, _rank_of_target

__all__ = ["reciprocal_rank"]


@torch.inference_mode()
def reciprocal_rank(
    input: torch.Tensor, target: torch.Tensor, *, k: Optional[int] = None
) -> torch.Tensor:
    """Per-sample 1 / (rank of target + 1), 0 beyond top-k.  Class: ``ReciprocalRank``."""
    return _reciprocal_rank(input, target, k, None)


def _reciprocal_rank(input: torch.Tensor, target: torch.Tensor, k: Optional[int], err: Optional[torch.Tensor]) -> torch.Tensor:
    """``reciprocal_rank`` with the class metric's device error flag (``err``, or None for the
    functional's own)."""
    _rank_input_check(input, target)
    out = _native_rank_scores(input, target, 1, k, err)
    if out is not None:
        return out
    rank = _rank_of_target(input, target)
    score = torch.reciprocal(rank + 1.0)
    if k is not None:
        score[rank >= k] = 0.0
    return score
