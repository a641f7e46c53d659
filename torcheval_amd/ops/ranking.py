"""Python wrapper of the K10 rank-of-target kernel (csrc/kernels/ranking.hip)."""

from typing import Optional

import torch

from torcheval_amd.ops import native, use_native

_SCORE_DTYPES = (torch.float32, torch.bfloat16, torch.float16)
_LABEL_DTYPES = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8)

HIT, RECIPROCAL = 0, 1


def native_rank(input: torch.Tensor, target: torch.Tensor) -> bool:
    """Whether K10 handles (input [N, C] scores, target [N] class indices) on this device."""
    return (
        use_native(input)
        and target.is_cuda
        and input.dim() == 2
        and target.dim() == 1
        and input.dtype in _SCORE_DTYPES
        and target.dtype in _LABEL_DTYPES
    )


def rank_scores(
    input: torch.Tensor, target: torch.Tensor, mode: int, k: Optional[int], err: Optional[torch.Tensor] = None
) -> torch.Tensor:
    """float32 [N]: ``mode=HIT`` -> 1.0 where rank(target) < k; ``mode=RECIPROCAL`` ->
    1 / (rank + 1), 0 where rank >= k (``k=None``: no cutoff).  rank = #{j : input[i, j] >
    input[i, target[i]]}.  Rows with an out-of-range target score NaN and set ``err``."""
    return native().rank_scores(input, target, mode, 0 if k is None else int(k), err)
