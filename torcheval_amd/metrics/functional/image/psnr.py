"""Peak signal-to-noise ratio, functional API (parity: functional/image/psnr.py)."""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import rowsums as _rs

__all__ = ["peak_signal_noise_ratio"]


@torch.inference_mode()
def peak_signal_noise_ratio(
    input: torch.Tensor, target: torch.Tensor, data_range: Optional[float] = None
) -> torch.Tensor:
    """PSNR = 10 log10(range^2 / MSE); ``data_range`` defaults to target max - min.
    Class version: ``PeakSignalNoiseRatio``."""
    _psnr_param_check(data_range)
    fused = _psnr_fused(input, target, data_range)
    if fused is not None:
        return fused
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


def _psnr_fused(input: torch.Tensor, target: torch.Tensor, data_range: Optional[float]) -> Optional[torch.Tensor]:
    """K5b: SSE, count and (auto range) target min / max in one launch, then the reference's
    compute.  Only where every intermediate keeps the reference's dtype (f32 / f64 inputs of
    one dtype); anything else returns None (ATen path)."""
    if input.dtype != target.dtype or input.dtype not in (torch.float32, torch.float64):
        return None
    if input.shape != target.shape or not _rs.supported(input, target):
        return None
    buf = torch.empty(4, dtype=input.dtype, device=input.device)
    outs = [(buf[0], _rs.SSE, _rs.SET), (buf[1], _rs.COUNT, _rs.SET)]
    if data_range is None:
        outs += [(buf[2], _rs.TMIN, _rs.SET), (buf[3], _rs.TMAX, _rs.SET)]
    _rs.update_states(input, target, None, outs)
    rng = buf[3] - buf[2] if data_range is None else torch.tensor(data=data_range, device=target.device)
    return _psnr_compute(buf[0], buf[1], rng)
