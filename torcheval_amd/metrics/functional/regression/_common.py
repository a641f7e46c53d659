"""K5 weighted-sums dispatch shared by the regression metrics."""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import use_native


def _native(input: torch.Tensor, target: torch.Tensor, w: Optional[torch.Tensor] = None) -> bool:
    from torcheval_amd.ops.reductions import moments_supported

    return use_native(input) and moments_supported(input, target, w) and input.numel() > 0


def _update(
    input: torch.Tensor, target: torch.Tensor, sample_weight: Optional[torch.Tensor]
) -> Tuple[torch.Tensor, torch.Tensor]:
    squared_error = torch.square(target - input)
    if sample_weight is None:
        return squared_error.sum(dim=0), torch.tensor(target.size(0), device=target.device)
    if squared_error.ndim == 2:
        sample_weight = sample_weight.unsqueeze(-1)
    return (squared_error * sample_weight).sum(dim=0), sample_weight.sum(dim=0).squeeze()
