"""Weighted sum, functional API (parity: functional/aggregation/sum.py)."""

from typing import Union

import torch

from torcheval_amd.ops import rowsums as _rs

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
    out_dtype = torch.result_type(input, weight) if isinstance(weight, (torch.Tensor, float, int)) else None
    if out_dtype in (torch.float32, torch.float64) and _rs.weight_ok(input, weight) and _rs.supported(
        input, weight if isinstance(weight, torch.Tensor) else None
    ):
        out = torch.empty((), dtype=out_dtype, device=input.device)
        _rs.update_states(input, None, weight, [(out, _rs.WX, _rs.SET)])  # K5b: one launch
        return out
    return _sum_update(input, weight)
