"""Small tensor helpers (parity: functional/tensor_utils.py:12-33)."""

from typing import List, Union

import torch


def _riemann_integral(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Left Riemann sum of y over the (descending) x grid: -sum((x[1:] - x[:-1]) * y[:-1])."""
    return -torch.sum((x[1:] - x[:-1]) * y[:-1])


def _create_threshold_tensor(
    threshold: Union[int, List[float], torch.Tensor], device: torch.device
) -> torch.Tensor:
    """An int n becomes ``linspace(0, 1, n)``; a list becomes a tensor; tensors pass through."""
    if isinstance(threshold, int):
        return torch.linspace(0, 1.0, threshold, device=device)
    if isinstance(threshold, list):
        return torch.tensor(threshold, device=device)
    return threshold
