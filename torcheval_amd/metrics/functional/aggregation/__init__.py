"""Aggregation metrics, functional API (parity: functional/aggregation/{auc,mean,sum,throughput}.py)."""

from torcheval_amd.metrics.functional.aggregation.auc import (
    _auc_compute,
    _auc_update_input_check,
    auc,
)
from torcheval_amd.metrics.functional.aggregation.mean import _mean_update, _mean_compute, mean
from torcheval_amd.metrics.functional.aggregation.sum import _sum_update, sum
from torcheval_amd.metrics.functional.aggregation.throughput import _throughput_compute, throughput

__all__ = [
    "auc",
    "mean",
    "sum",
    "throughput",
]
__doc_name__ = "Aggregation Metrics"
