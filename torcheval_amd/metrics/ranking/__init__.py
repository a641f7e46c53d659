"""Ranking class metrics (parity: metrics/ranking/*.py)."""

from torcheval_amd.metrics.ranking._score_list import _ScoreList, _RankScoreList
from torcheval_amd.metrics.ranking.click_through_rate import ClickThroughRate
from torcheval_amd.metrics.ranking.hit_rate import HitRate
from torcheval_amd.metrics.ranking.reciprocal_rank import ReciprocalRank
from torcheval_amd.metrics.ranking.retrieval_precision import RetrievalPrecision
from torcheval_amd.metrics.ranking.weighted_calibration import WeightedCalibration

__all__ = [
    "ClickThroughRate",
    "HitRate",
    "ReciprocalRank",
    "RetrievalPrecision",
    "WeightedCalibration",
]
__doc_name__ = "Ranking Metrics"
