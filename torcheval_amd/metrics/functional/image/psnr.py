"""Peak signal-to-noise ratio, functional API (parity: functional/image/psnr.py)."""

from typing import Optional, Tuple

import torch

__all__ = ["peak_signal_noise_ratio"]


@torch.inference_mode()
def peak_signal_noise_ratio(
    input: torch.Tensor, target: torch.Tensor, data_range: Optional[float] = None
) -> torch.Tensor:
    """PSNR = 10 log10(range^2 / MSE); ``data_range`` defaults to target max - min.
    Class version: ``PeakSignalNoiseRatio``."""
    _psnr_param_check(data_range)
    if data_range is None:
        data_range_tensor = torch.max(target) - torch.min(target)
    else:
        data_range_tensor = torch.tensor(data=data_range, device=target.device)
    sse, n = _psnr_update(input, target)
    return _psnr_compute(sse, n, data_range_tensor)


def _psnr_param_check(data_range: Optional[float]) -> None:
    if data_range is not None:
        if type(data_range) is not float:
            raise ValueError("`data_range needs to be either `None` or `float`.")
        if data_range <= 0:
            raise ValueError("`data_range` needs to be positive.")


def _psnr_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.shape != target.shape:
        raise ValueError(
            f"The `input` and `target` must have the same shape, got shapes {input.shape} and {target.shape}."
        )


def _psnr_update(input: torch.Tensor, target: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    _psnr_input_check(input, target)
    return torch.sum(torch.pow(input - target, 2)), torch.tensor(target.numel(), device=target.device)


def _psnr_compute(sum_square_error: torch.Tensor, num_observations: torch.Tensor, data_range: torch.Tensor) -> torch.Tensor:
    mse = sum_square_error / num_observations
    return 10 * torch.log10(torch.pow(data_range, 2) / mse)
