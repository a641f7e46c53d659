from torcheval_amd.utils.test_utils.dist_pool import run_distributed
from torcheval_amd.utils.test_utils.dummy_metric import (
    DummySumDictStateMetric,
    DummySumListStateMetric,
    DummySumMetric,
)
from torcheval_amd.utils.test_utils.metric_class_tester import assert_result_close, MetricClassTester

__all__ = [
    "DummySumDictStateMetric",
    "DummySumListStateMetric",
    "DummySumMetric",
    "MetricClassTester",
    "assert_result_close",
    "run_distributed",
]
