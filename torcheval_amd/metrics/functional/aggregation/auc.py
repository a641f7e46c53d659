"""Trapezoidal AUC, functional API (parity: functional/aggregation/auc.py).

ROCm float32 with ``reorder=True`` (the class metric's default): K3a's ascending stable radix
sort carries y through as its payload (no ``gather``) and K3t (csrc/kernels/trapz.hip) sums the
trapezoids per task in FP64 - instead of torch.sort(stable) + gather + trapz.  The ATen form
below stays the CPU path and the oracle of the GPU tests.
"""

from typing import Optional

import torch

from torcheval_amd.ops import use_native

__all__ = ["auc"]

_Y_DTYPES = (torch.float32, torch.int64, torch.int32, torch.uint8, torch.bool)


def _auc_native(x: torch.Tensor, y: torch.Tensor) -> Optional[torch.Tensor]:
    """float32 [tasks] areas of the x-sorted pairs, or None when the native path does not apply."""
    # y rides K3a's target payload, converted to its f32 value (as trapz's float32 promotion does)
    if not (use_native(x) and x.dtype == torch.float32 and y.dtype in _Y_DTYPES and y.device == x.device
            and x.shape == y.shape and x.shape[-1] < 2**31):
        return None
    from torcheval_amd.ops import native
    from torcheval_amd.ops.sortscan import PAYLOAD_TARGET

    xs = x.contiguous()
    s = torch.empty(xs.shape, dtype=torch.float32, device=x.device)
    order = torch.empty(xs.shape, dtype=torch.int32, device=x.device)
    native().sort_desc(xs, s, order, y.contiguous(), PAYLOAD_TARGET, None, True)  # ascending, stable
    out = torch.empty(xs.shape[0], dtype=torch.float32, device=x.device)
    native().trapz_sorted(s, order, out)
    return out


def _auc_compute(x: torch.Tensor, y: torch.Tensor, reorder: bool = False) -> torch.Tensor:
    if x.numel() == 0 or y.numel() == 0:
        return torch.tensor([])
    if x.ndim == 1:
        x = x.unsqueeze(0)
    if y.ndim == 1:
        y = y.unsqueeze(0)
    if reorder:
        out = _auc_native(x, y)
        if out is not None:
            return out
        x, idx = torch.sort(x, dim=1, stable=True)
        y = y.gather(1, idx)
    return torch.trapz(y, x)


def _auc_update_input_check(x: torch.Tensor, y: torch.Tensor, n_tasks: int = 1) -> None:
    size_x, size_y = x.size(), y.size()
    if x.ndim == 1:
        x = x.unsqueeze(0)
    if y.ndim == 1:
        y = y.unsqueeze(0)
    if x.numel() == 0 or y.numel() == 0:
        raise ValueError(
            f"The `x` and `y` should have atleast 1 element, got shapes {size_x} and {size_y}."
        )
    if x.size() != y.size():
        raise ValueError(
            f"Expected the same shape in `x` and `y` tensor but got shapes {size_x} and {size_y}."
        )
    if x.size(0) != n_tasks or y.size(0) != n_tasks:
        raise ValueError(
            f"Expected `x` dim_1={x.size(0)} and `y` dim_1={y.size(0)} have first dimension equals to n_tasks={n_tasks}."
        )


def auc(x: torch.Tensor, y: torch.Tensor, reorder: bool = False) -> torch.Tensor:
    """Trapezoidal area under the curve y(x) per task (``[n]`` or ``[n_tasks, n]``).
    Class version: ``torcheval_amd.metrics.AUC``."""
    n_tasks = x.size(0) if x.ndim > 1 else 1
    _auc_update_input_check(x, y, n_tasks)
    return _auc_compute(x, y, reorder)
