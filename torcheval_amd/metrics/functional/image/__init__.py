"""Image metrics, functional API (parity: functional/image/psnr.py)."""

from torcheval_amd.metrics.functional.image.psnr import (
    peak_signal_noise_ratio,
    _psnr_param_check,
    _psnr_input_check,
    _psnr_update,
    _psnr_compute,
)

__all__ = [
    "peak_signal_noise_ratio",
]
__doc_name__ = "Image Metrics"
