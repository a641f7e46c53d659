"""Regression class metrics (parity: metrics/regression/*.py)."""

from torcheval_amd.metrics.regression.mean_squared_error import MeanSquaredError
from torcheval_amd.metrics.regression.r2_score import R2Score

__all__ = [
    "MeanSquaredError",
    "R2Score",
]
__doc_name__ = "Regression Metrics"
