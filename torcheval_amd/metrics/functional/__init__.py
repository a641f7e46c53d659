"""Functional (stateless) metrics — parity with torcheval/metrics/functional/__init__.py."""

from torcheval_amd.metrics.functional.classification import *  # noqa: F401,F403
from torcheval_amd.metrics.functional.classification import __all__ as _cls_all

__all__ = list(_cls_all)
