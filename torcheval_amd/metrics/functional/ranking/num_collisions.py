"""Number of collisions, functional API (parity: functional/ranking/num_collisions.py)."""

import torch

__all__ = ["num_collisions"]


@torch.inference_mode()
def num_collisions(input: torch.Tensor) -> torch.Tensor:
    """For every element, how many OTHER elements hold the same (integer) id."""
    if input.ndim != 1:
        raise ValueError(f"input should be a one-dimensional tensor, got shape {input.shape}.")
    if input.dtype not in (torch.int, torch.int8, torch.int16, torch.int32, torch.int64):
        raise ValueError(f"input should be an integer tensor, got {input.dtype}.")
    _, inverse, counts = torch.unique(input, return_inverse=True, return_counts=True)
    return counts[inverse] - 1
