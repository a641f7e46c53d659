"""Ranking metrics, functional API (parity: functional/ranking/*.py).

``num_collisions`` is O(N log N) (sort + run lengths) instead of the reference's N x N
equality matrix (num_collisions.py:32-36).
"""

from typing import Optional, Tuple, Union

import torch

__all__ = [
    "click_through_rate",
    "frequency_at_k",
    "hit_rate",
    "num_collisions",
    "reciprocal_rank",
    "weighted_calibration",
    "retrieval_precision",
]
__doc_name__ = "Ranking Metrics"


# ----------------------------------------------------------------------------- CTR
@torch.inference_mode()
def click_through_rate(
    input: torch.Tensor, weights: Optional[torch.Tensor] = None, *, num_tasks: int = 1
) -> torch.Tensor:
    """Weighted fraction of clicks per task.  Class version: ``ClickThroughRate``."""
    if weights is None:
        weights = 1.0
    click_total, weight_total = _click_through_rate_update(input, weights, num_tasks=num_tasks)
    return _click_through_rate_compute(click_total, weight_total)


def _click_through_rate_update(
    input: torch.Tensor, weights: Union[torch.Tensor, float, int] = 1.0, *, num_tasks: int
) -> Tuple[torch.Tensor, torch.Tensor]:
    _click_through_rate_input_check(input, weights, num_tasks=num_tasks)
    if isinstance(weights, torch.Tensor):
        weights = weights.type(torch.float)
        return (input * weights).sum(-1), weights.sum(-1)
    click_total = weights * input.sum(-1).type(torch.float)
    return click_total, weights * input.size(-1) * torch.ones_like(click_total)


def _click_through_rate_compute(click_total: torch.Tensor, weight_total: torch.Tensor) -> torch.Tensor:
    return click_total / (weight_total + torch.finfo(weight_total.dtype).tiny)


def _click_through_rate_input_check(
    input: torch.Tensor, weights: Union[torch.Tensor, float, int], *, num_tasks: int
) -> None:
    if input.ndim != 1 and input.ndim != 2:
        raise ValueError(f"`input` should be a one or two dimensional tensor, got shape {input.shape}.")
    if isinstance(weights, torch.Tensor) and weights.shape != input.shape:
        raise ValueError(
            "tensor `weights` should have the same shape as tensor `input`, "
            f"got shapes {weights.shape} and {input.shape}, respectively."
        )
    _num_tasks_check(input, num_tasks)


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


# ----------------------------------------------------------------------------- frequency
@torch.inference_mode()
def frequency_at_k(input: torch.Tensor, k: float) -> torch.Tensor:
    """Indicator of ``input < k`` (e.g. feature frequency below a cutoff)."""
    if input.ndim != 1:
        raise ValueError(f"input should be a one-dimensional tensor, got shape {input.shape}.")
    if k < 0:
        raise ValueError(f"k should not be negative, got {k}.")
    return (input < k).float()


# ----------------------------------------------------------------------------- rank based
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


@torch.inference_mode()
def hit_rate(
    input: torch.Tensor, target: torch.Tensor, *, k: Optional[int] = None, _err: Optional[torch.Tensor] = None
) -> torch.Tensor:
    """Per-sample 1.0 if the target is within the top-k scores.  Class: ``HitRate``."""
    _rank_input_check(input, target)
    if k is not None and k <= 0:
        raise ValueError(f"k should be None or positive, got {k}.")
    if k is None or k >= input.size(dim=-1):
        return input.new_ones(target.size())
    out = _native_rank_scores(input, target, 0, k, _err)
    if out is not None:
        return out
    return (_rank_of_target(input, target) < k).float()


@torch.inference_mode()
def reciprocal_rank(
    input: torch.Tensor, target: torch.Tensor, *, k: Optional[int] = None, _err: Optional[torch.Tensor] = None
) -> torch.Tensor:
    """Per-sample 1 / (rank of target + 1), 0 beyond top-k.  Class: ``ReciprocalRank``."""
    _rank_input_check(input, target)
    out = _native_rank_scores(input, target, 1, k, _err)
    if out is not None:
        return out
    rank = _rank_of_target(input, target)
    score = torch.reciprocal(rank + 1.0)
    if k is not None:
        score[rank >= k] = 0.0
    return score


# ----------------------------------------------------------------------------- collisions
@torch.inference_mode()
def num_collisions(input: torch.Tensor) -> torch.Tensor:
    """For every element, how many OTHER elements hold the same (integer) id."""
    if input.ndim != 1:
        raise ValueError(f"input should be a one-dimensional tensor, got shape {input.shape}.")
    if input.dtype not in (torch.int, torch.int8, torch.int16, torch.int32, torch.int64):
        raise ValueError(f"input should be an integer tensor, got {input.dtype}.")
    _, inverse, counts = torch.unique(input, return_inverse=True, return_counts=True)
    return counts[inverse] - 1


# ----------------------------------------------------------------------------- calibration
@torch.inference_mode()
def weighted_calibration(
    input: torch.Tensor,
    target: torch.Tensor,
    weight: Union[float, int, torch.Tensor] = 1.0,
    *,
    num_tasks: int = 1,
) -> torch.Tensor:
    """sum(w * input) / sum(w * target) per task.  Class: ``WeightedCalibration``."""
    wi, wt = _weighted_calibration_update(input, target, weight, num_tasks=num_tasks)
    return wi / wt


def _weighted_calibration_update(
    input: torch.Tensor,
    target: torch.Tensor,
    weight: Union[float, int, torch.Tensor],
    *,
    num_tasks: int,
) -> Tuple[torch.Tensor, torch.Tensor]:
    if input.shape != target.shape:
        raise ValueError(f"`input` shape ({input.shape}) is different from `target` shape ({target.shape})")
    _num_tasks_check(input, num_tasks)
    if isinstance(weight, (float, int)):
        return weight * torch.sum(input, dim=-1), weight * torch.sum(target, dim=-1)
    if isinstance(weight, torch.Tensor) and input.size() == weight.size():
        return torch.sum(weight * input, dim=-1), torch.sum(weight * target, dim=-1)
    raise ValueError(
        "Weight must be either a float value or a tensor that matches the input tensor size. "
        f"Got {weight} instead."
    )


# ----------------------------------------------------------------------------- retrieval
@torch.inference_mode()
def retrieval_precision(
    input: torch.Tensor,
    target: torch.Tensor,
    k: Optional[int] = None,
    limit_k_to_size: bool = False,
    num_tasks: int = 1,
) -> torch.Tensor:
    """Fraction of relevant items among the top-k scored ones.  Class: ``RetrievalPrecision``."""
    _retrieval_precision_param_check(k, limit_k_to_size)
    _retrieval_precision_update_input_check(input, target, num_tasks)
    return _retrieval_precision_compute(input, target, k, limit_k_to_size)


def _retrieval_precision_param_check(k: Optional[int] = None, limit_k_to_size: bool = False) -> None:
    if k is not None and k <= 0:
        raise ValueError(f"k must be a positive integer, got k={k}.")
    if limit_k_to_size and k is None:
        raise ValueError("when limit_k_to_size is True, k must be a positive (>0) integer.")


def _retrieval_precision_update_input_check(
    input: torch.Tensor,
    target: torch.Tensor,
    num_tasks: int = 1,
    indexes: Optional[torch.Tensor] = None,
    num_queries: int = 1,
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            f"input and target must be of the same shape, got input.shape={input.shape} and target.shape={target.shape}."
        )
    if num_tasks == 1:
        if input.dim() != 1:
            raise ValueError(
                f"input and target should be one dimensional tensors, got input and target dimensions={input.dim()}."
            )
    elif input.dim() != 2 or input.shape[0] != num_tasks:
        raise ValueError(
            f"input and target should be two dimensional tensors with {num_tasks} rows, got input and target shape={input.shape}."
        )


def get_topk(t: torch.Tensor, k: Optional[int]) -> Tuple[torch.Tensor, torch.Tensor]:
    n = t.size(-1)
    return t.topk(min(k if k is not None else n, n), dim=-1)


def compute_nb_relevant_items_retrieved(input: torch.Tensor, k: Optional[int], target: torch.Tensor) -> torch.Tensor:
    return target.gather(dim=-1, index=get_topk(input, k)[1]).sum(dim=-1)


def compute_total_number_items_retrieved(
    input: torch.Tensor, k: Optional[int] = None, limit_k_to_size: bool = False
) -> int:
    n = input.size(-1)
    if k is None:
        return n
    return min(k, n) if limit_k_to_size else k


def _retrieval_precision_compute(
    input: torch.Tensor, target: torch.Tensor, k: Optional[int] = None, limit_k_to_size: bool = False
) -> torch.Tensor:
    return compute_nb_relevant_items_retrieved(input, k, target) / compute_total_number_items_retrieved(
        input, k, limit_k_to_size
    )
