"""Aggregation class metrics (parity: metrics/aggregation/*.py)."""

from torcheval_amd.metrics.aggregation.auc import AUC
from torcheval_amd.metrics.aggregation.cat import Cat
from torcheval_amd.metrics.aggregation.max import Max
from torcheval_amd.metrics.aggregation.min import Min
from torcheval_amd.metrics.aggregation.mean import Mean
from torcheval_amd.metrics.aggregation.sum import Sum
from torcheval_amd.metrics.aggregation.throughput import Throughput

__all__ = [
    "AUC",
    "Cat",
    "Max",
    "Mean",
    "Min",
    "Sum",
    "Throughput",
]
__doc_name__ = "Aggregation Metrics"
