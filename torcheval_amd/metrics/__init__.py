"""Class (stateful) metrics — parity with torcheval/metrics/__init__.py.

``FrechetInceptionDistance`` resolves lazily (it pulls in the Inception-v3 model)."""

from torcheval_amd.metrics import functional
from torcheval_amd.metrics.aggregation import AUC, Cat, Max, Mean, Min, Sum, Throughput
from torcheval_amd.metrics.classification import *  # noqa: F401,F403
from torcheval_amd.metrics.classification import __all__ as _cls_all
from torcheval_amd.metrics.image import PeakSignalNoiseRatio
from torcheval_amd.metrics.metric import Metric
from torcheval_amd.metrics.ranking import (
    ClickThroughRate,
    HitRate,
    ReciprocalRank,
    RetrievalPrecision,
    WeightedCalibration,
)
from torcheval_amd.metrics.regression import MeanSquaredError, R2Score
from torcheval_amd.metrics.text import (
    BLEUScore,
    Perplexity,
    WordErrorRate,
    WordInformationLost,
    WordInformationPreserved,
)
from torcheval_amd.metrics.window import (
    WindowedBinaryAUROC,
    WindowedBinaryNormalizedEntropy,
    WindowedClickThroughRate,
    WindowedMeanSquaredError,
    WindowedWeightedCalibration,
)

__all__ = ["Metric", "functional"] + sorted(
    list(_cls_all)
    + ["AUC", "Cat", "Max", "Mean", "Min", "Sum", "Throughput"]
    + ["FrechetInceptionDistance", "PeakSignalNoiseRatio"]
    + ["ClickThroughRate", "HitRate", "ReciprocalRank", "RetrievalPrecision", "WeightedCalibration"]
    + ["MeanSquaredError", "R2Score"]
    + ["BLEUScore", "Perplexity", "WordErrorRate", "WordInformationLost", "WordInformationPreserved"]
    + ["WindowedBinaryAUROC", "WindowedBinaryNormalizedEntropy", "WindowedClickThroughRate"]
    + ["WindowedMeanSquaredError", "WindowedWeightedCalibration"]
)


def __getattr__(name):
    if name == "FrechetInceptionDistance":
        from torcheval_amd.metrics.image.fid import FrechetInceptionDistance

        return FrechetInceptionDistance
    raise AttributeError(name)
