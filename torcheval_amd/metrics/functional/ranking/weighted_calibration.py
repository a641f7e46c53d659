"""Weighted calibration, functional API (parity: functional/ranking/weighted_calibration.py)."""

from typing import Tuple, Union

import torch

from torcheval_amd.metrics.functional.ranking._rank_common import _num_tasks_check

__all__ = ["weighted_calibration"]


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
