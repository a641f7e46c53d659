"""Shared input checks and the K10 rank-of-target dispatch for the ranking metrics."""

from typing import Optional

import torch


def _num_tasks_check(input: torch.Tensor, num_tasks: int) -> None:
    if num_tasks == 1:
        if len(input.shape) > 1:
            raise ValueError(
                f"`num_tasks = 1`, `input` is expected to be one-dimensional tensor, but got shape ({input.shape})."
            )
    elif len(input.shape) == 1 or input.shape[0] != num_tasks:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input`'s shape is expected to be ({num_tasks}, num_samples), but got shape ({input.shape})."
        )


def _rank_of_target(input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    y_score = torch.gather(input, dim=-1, index=target.unsqueeze(dim=-1))
    return torch.gt(input, y_score).sum(dim=-1)


def _rank_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if target.ndim != 1:
        raise ValueError(f"target should be a one-dimensional tensor, got shape {target.shape}.")
    if input.ndim != 2:
        raise ValueError(f"input should be a two-dimensional tensor, got shape {input.shape}.")
    if input.shape[0] != target.shape[0]:
        raise ValueError(
            "`input` and `target` should have the same minibatch dimension, ",
            f"got shapes {input.shape} and {target.shape}, respectively.",
        )


def _native_rank_scores(input, target, mode: int, k: Optional[int], err: Optional[torch.Tensor]):
    """K10 (one streaming pass, no [N, C] temporaries) when the tensors are on a ROCm device.
    Out-of-range targets are recorded in ``err`` (class path: raised at ``compute()``) or, for
    the functional call without ``err``, raised here when ``config.validate`` is on; otherwise
    their rows score NaN."""
    from torcheval_amd.config import config
    from torcheval_amd.ops.ranking import native_rank, rank_scores

    if not native_rank(input, target):
        return None
    own = err is None and config.validate
    if own:
        err = torch.zeros(1, dtype=torch.int32, device=input.device)
    out = rank_scores(input, target, mode, k, err)
    if own:
        from torcheval_amd.metrics.classification.accuracy import _raise_on_device_error

        _raise_on_device_error(err)
    return out
