"""Windowed metrics (parity: metrics/window/__init__.py)."""

from torcheval_amd.metrics.window.auroc import WindowedBinaryAUROC
from torcheval_amd.metrics.window.click_through_rate import WindowedClickThroughRate
from torcheval_amd.metrics.window.mean_squared_error import WindowedMeanSquaredError
from torcheval_amd.metrics.window.normalized_entropy import WindowedBinaryNormalizedEntropy
from torcheval_amd.metrics.window.weighted_calibration import WindowedWeightedCalibration

__all__ = [
    "WindowedBinaryAUROC",
    "WindowedBinaryNormalizedEntropy",
    "WindowedClickThroughRate",
    "WindowedMeanSquaredError",
    "WindowedWeightedCalibration",
]
__doc_name__ = "Windowed Metrics"
