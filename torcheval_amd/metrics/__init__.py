"""Class (stateful) metrics — parity with torcheval/metrics/__init__.py."""

from torcheval_amd.metrics.classification import *  # noqa: F401,F403
from torcheval_amd.metrics.classification import __all__ as _cls_all
from torcheval_amd.metrics.metric import Metric

__all__ = ["Metric"] + list(_cls_all)
