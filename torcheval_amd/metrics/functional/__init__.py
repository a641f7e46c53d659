"""Functional (stateless) metrics — parity with torcheval/metrics/functional/__init__.py."""

from torcheval_amd.metrics.functional.aggregation import auc, mean, sum, throughput
from torcheval_amd.metrics.functional.classification import *  # noqa: F401,F403
from torcheval_amd.metrics.functional.classification import __all__ as _cls_all
from torcheval_amd.metrics.functional.image import peak_signal_noise_ratio
from torcheval_amd.metrics.functional.ranking import (
    click_through_rate,
    frequency_at_k,
    hit_rate,
    num_collisions,
    reciprocal_rank,
    retrieval_precision,
    weighted_calibration,
)
from torcheval_amd.metrics.functional.regression import mean_squared_error, r2_score
from torcheval_amd.metrics.functional.text import (
    bleu_score,
    perplexity,
    word_error_rate,
    word_information_lost,
    word_information_preserved,
)

__all__ = sorted(
    list(_cls_all)
    + ["auc", "mean", "sum", "throughput", "peak_signal_noise_ratio"]
    + ["click_through_rate", "frequency_at_k", "hit_rate", "num_collisions", "reciprocal_rank"]
    + ["retrieval_precision", "weighted_calibration", "mean_squared_error", "r2_score"]
    + ["bleu_score", "perplexity", "word_error_rate", "word_information_lost"]
    + ["word_information_preserved"]
)
