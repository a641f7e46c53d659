"""Frequency at k, functional API (parity: functional/ranking/frequency.py)."""

import torch

__all__ = ["frequency_at_k"]


@torch.inference_mode()
def frequency_at_k(input: torch.Tensor, k: float) -> torch.Tensor:
    """Indicator of ``input < k`` (e.g. feature frequency below a cutoff)."""
    if input.ndim != 1:
        raise ValueError(f"input should be a one-dimensional tensor, got shape {input.shape}.")
    if k < 0:
        raise ValueError(f"k should not be negative, got {k}.")
    return (input < k).float()
