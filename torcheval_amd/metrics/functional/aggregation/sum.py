"""Weighted sum, functional API (parity: functional/aggregation/sum.py)."""

from typing import Union

import torch

__all__ = ["sum"]


def _sum_update(input: torch.Tensor, weight: Union[float, int, torch.Tensor]) -> torch.Tensor:
    if isinstance(weight, (float, int)) or (
        isinstance(weight, torch.Tensor) and input.size() == weight.size()
    ):
        return (input * weight).sum()
    raise ValueError(
        "Weight must be either a float value or an int value or a tensor that matches the input tensor size. "
        f"Got {weight} instead."
    )


@torch.inference_mode()
def sum(input: torch.Tensor, weight: Union[float, torch.Tensor] = 1.0) -> torch.Tensor:  # noqa: A001
    """Weighted sum.  Class version: ``torcheval_amd.metrics.Sum``."""
    return _sum_update(input, weight)
