"""Retrieval precision at k, functional API (parity: functional/ranking/retrieval_precision.py)."""

from typing import Optional, Tuple

import torch

__all__ = ["retrieval_precision", "get_topk", "compute_nb_relevant_items_retrieved", "compute_total_number_items_retrieved"]


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
