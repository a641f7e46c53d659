"""Weighted calibration, functional API (parity: functional/ranking/weighted_calibration.py)."""

from typing import Tuple, Union

import torch

from torcheval_amd.metrics.functional.ranking._rank_common import _num_tasks_check
from torcheval_amd.ops import rowsums as _rs

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
    if (input.dtype in (torch.float32, torch.float64) and target.dtype == input.dtype and input.shape == target.shape
            and _rs.weight_ok(input, weight) and (not isinstance(weight, torch.Tensor) or weight.dtype == input.dtype)
            and _rs.supported(input, target, weight if isinstance(weight, torch.Tensor) else None)):
        _num_tasks_check(input, num_tasks)
        rows = input.shape[0] if input.ndim == 2 else 1
        buf = torch.empty(2, rows, dtype=input.dtype, device=input.device)
        _rs.update_states(input, target, weight, [(buf[0], _rs.WX, _rs.SET), (buf[1], _rs.WT, _rs.SET)], rows=rows)
        wi, wt = (buf[0], buf[1]) if input.ndim == 2 else (buf[0, 0], buf[1, 0])
        return wi / wt  # K5b sums + one divide
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
