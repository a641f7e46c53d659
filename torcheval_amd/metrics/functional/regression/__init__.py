"""Regression metrics, functional API (parity: functional/regression/*.py)."""

from torcheval_amd.metrics.functional.regression._common import _native, _update
from torcheval_amd.metrics.functional.regression.mean_squared_error import (
    mean_squared_error,
    _mean_squared_error_update,
    _mean_squared_error_compute,
    _mean_squared_error_update_input_check,
    _mean_squared_error_param_check,
)
from torcheval_amd.metrics.functional.regression.r2_score import (
    r2_score,
    _r2_score_update,
    _r2_score_compute,
    _r2_score_param_check,
    _r2_score_update_input_check,
)

__all__ = [
    "mean_squared_error",
    "r2_score",
]
__doc_name__ = "Regression Metrics"
