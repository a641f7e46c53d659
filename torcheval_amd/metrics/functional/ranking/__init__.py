"""Ranking metrics, functional API (parity: functional/ranking/*.py)."""

from torcheval_amd.metrics.functional.ranking._rank_common import (
    _num_tasks_check,
    _rank_of_target,
    _rank_input_check,
    _native_rank_scores,
)
from torcheval_amd.metrics.functional.ranking.click_through_rate import (
    click_through_rate,
    _click_through_rate_update,
    _click_through_rate_compute,
    _click_through_rate_input_check,
)
from torcheval_amd.metrics.functional.ranking.frequency import frequency_at_k
from torcheval_amd.metrics.functional.ranking.hit_rate import hit_rate
from torcheval_amd.metrics.functional.ranking.reciprocal_rank import reciprocal_rank
from torcheval_amd.metrics.functional.ranking.num_collisions import num_collisions
from torcheval_amd.metrics.functional.ranking.weighted_calibration import (
    weighted_calibration,
    _weighted_calibration_update,
)
from torcheval_amd.metrics.functional.ranking.retrieval_precision import (
    retrieval_precision,
    _retrieval_precision_param_check,
    _retrieval_precision_update_input_check,
    get_topk,
    compute_nb_relevant_items_retrieved,
    compute_total_number_items_retrieved,
    _retrieval_precision_compute,
)

__all__ = [
    "click_through_rate",
    "frequency_at_k",
    "hit_rate",
    "num_collisions",
    "reciprocal_rank",
    "retrieval_precision",
    "weighted_calibration",
]
__doc_name__ = "Ranking Metrics"
