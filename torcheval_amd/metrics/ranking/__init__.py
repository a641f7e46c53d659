"""Ranking metrics, class API (parity: metrics/ranking/*.py)."""

from typing import Iterable, List, Optional, Union

import torch
from typing_extensions import Literal

from torcheval_amd.metrics.functional.ranking import (
    _click_through_rate_compute,
    _click_through_rate_update,
    _retrieval_precision_param_check,
    _retrieval_precision_update_input_check,
    _weighted_calibration_update,
    get_topk,
    hit_rate,
    reciprocal_rank,
    retrieval_precision,
)
from torcheval_amd.metrics.metric import Metric

__all__ = ["ClickThroughRate", "HitRate", "ReciprocalRank", "RetrievalPrecision", "WeightedCalibration"]
__doc_name__ = "Ranking Metrics"


class ClickThroughRate(Metric[torch.Tensor]):
    """Weighted click-through rate per task (float64 sums, ``merge="sum"``)."""

    def __init__(self, *, num_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        if num_tasks < 1:
            raise ValueError(
                "`num_tasks` value should be greater than and equal to 1, but received {num_tasks}. "
            )
        self.num_tasks = num_tasks
        for name in ("click_total", "weight_total"):
            self._add_state(name, torch.zeros(num_tasks, dtype=torch.float64, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, input: torch.Tensor, weights: Union[torch.Tensor, float, int] = 1.0) -> "ClickThroughRate":
        click_total, weight_total = _click_through_rate_update(input, weights, num_tasks=self.num_tasks)
        self.click_total = self.click_total + click_total
        self.weight_total = self.weight_total + weight_total
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _click_through_rate_compute(self.click_total, self.weight_total)

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["ClickThroughRate"]) -> "ClickThroughRate":
        for metric in metrics:
            self.click_total = self.click_total + metric.click_total.to(self.device)
            self.weight_total = self.weight_total + metric.weight_total.to(self.device)
        return self


class _ScoreList(Metric[torch.Tensor]):
    def __init__(self, *, k: Optional[int] = None, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self.k = k
        self._add_state("scores", [], merge="cat")

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if not self.scores:
            return torch.empty(0)
        return torch.cat(self.scores, dim=0)

    @torch.inference_mode()
    def merge_state(self, metrics):
        for metric in metrics:
            if metric.scores:
                self.scores.append(torch.cat(metric.scores).to(self.device))
        return self

    @torch.inference_mode()
    def _prepare_for_merge_state(self) -> None:
        if self.scores:
            self.scores = [torch.cat(self.scores)]


class _RankScoreList(_ScoreList):
    """ROCm inputs run K10; out-of-range targets land in a device flag raised at ``compute()``."""

    _err: Optional[torch.Tensor] = None

    def _err_for(self, input: torch.Tensor) -> Optional[torch.Tensor]:
        if not input.is_cuda:
            return None
        if self._err is None or self._err.device != input.device:
            self._err = torch.zeros(1, dtype=torch.int32, device=input.device)
        return self._err

    def _check_device_errors(self) -> None:
        from torcheval_amd.metrics.classification.accuracy import _raise_on_device_error

        _raise_on_device_error(self._err)

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        self._check_device_errors()
        return super().compute()


class HitRate(_RankScoreList):
    """Per-sample hit (target within top-k) scores, concatenated over updates."""

    @torch.inference_mode()
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "HitRate":
        self.scores.append(hit_rate(input, target, k=self.k, _err=self._err_for(input)))
        return self


class ReciprocalRank(_RankScoreList):
    """Per-sample reciprocal rank scores, concatenated over updates."""

    @torch.inference_mode()
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "ReciprocalRank":
        self.scores.append(reciprocal_rank(input, target, k=self.k, _err=self._err_for(input)))
        return self


class RetrievalPrecision(Metric[torch.Tensor]):
    """
    Precision@k per query with a bounded-memory streaming top-k per query.

    Args:
        empty_target_action: result for a query without positives: "neg" (0), "pos" (1),
            "skip" (NaN) or "err" (raise).
        k, limit_k_to_size: cutoff and whether it is clipped to the number of items.
        num_queries: number of queries (``indexes`` selects the query of each sample).
        avg: None (per query) or "macro" (nan-mean over queries).
    """

    def __init__(
        self,
        empty_target_action: Union[Literal["neg"], Literal["pos"], Literal["skip"], Literal["err"]] = "neg",
        k: Optional[int] = None,
        limit_k_to_size: bool = False,
        num_queries: int = 1,
        avg: Optional[Union[Literal["macro"], Literal["none"]]] = None,
        device: Optional[torch.device] = None,
    ) -> None:
        _retrieval_precision_param_check(k, limit_k_to_size)
        super().__init__(device=device)
        self.empty_target_action = empty_target_action
        self.num_queries = num_queries
        self.k = k
        self.limit_k_to_size = limit_k_to_size
        self.avg = avg
        self._add_state("topk", [torch.empty(0, device=self.device) for _ in range(num_queries)])
        self._add_state("target", [torch.empty(0, device=self.device) for _ in range(num_queries)])

    @torch.inference_mode()
    def update(
        self, input: torch.Tensor, target: torch.Tensor, indexes: Optional[torch.Tensor] = None
    ) -> "RetrievalPrecision":
        _retrieval_precision_update_input_check(input, target, num_queries=self.num_queries, indexes=indexes)
        if self.num_queries == 1:
            self.update_single_query(0, input, target)
            return self
        if indexes is None:
            raise ValueError("`indexes` must be passed during update() when num_queries > 1.")
        # one host sync for the set of present queries (reference: one `i in indexes` per query)
        for i in torch.unique(indexes).tolist():
            if 0 <= i < self.num_queries:
                sel = indexes == i
                self.update_single_query(int(i), input[sel], target[sel])
        return self

    def update_single_query(self, i: int, input: torch.Tensor, target: torch.Tensor) -> None:
        preds = torch.cat([self.topk[i].to(input.device, input.dtype), input])
        targets = torch.cat([self.target[i].to(target.device, target.dtype), target])
        values, idx = get_topk(preds, self.k)
        self.topk[i] = values
        self.target[i] = targets.gather(dim=-1, index=idx)

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        rp: List[torch.Tensor] = []
        for i in range(self.num_queries):
            tgt = self.target[i]
            if not len(tgt):
                rp.append(torch.tensor([torch.nan]))
            elif not bool((tgt == 1).any()):
                if self.empty_target_action == "pos":
                    rp.append(torch.tensor([1.0]))
                elif self.empty_target_action == "neg":
                    rp.append(torch.tensor([0.0]))
                elif self.empty_target_action == "skip":
                    rp.append(torch.tensor([torch.nan]))
                elif self.empty_target_action == "err":
                    raise ValueError(f"no positive value found in target={tgt.float()}.")
            else:
                rp.append(
                    retrieval_precision(self.topk[i], tgt, self.k, self.limit_k_to_size).reshape(-1).cpu()
                )
        out = torch.cat(rp).to(self.device)
        return out.nanmean() if self.avg == "macro" else out

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["RetrievalPrecision"]) -> "RetrievalPrecision":
        metrics = list(metrics)
        for i in range(self.num_queries):
            self.topk[i] = torch.cat([self.topk[i]] + [m.topk[i].to(self.device) for m in metrics]).to(self.device)
            self.target[i] = torch.cat([self.target[i]] + [m.target[i].to(self.device) for m in metrics]).to(self.device)
        return self


class WeightedCalibration(Metric[torch.Tensor]):
    """sum(w * input) / sum(w * target) per task (float64 sums, ``merge="sum"``)."""

    def __init__(self, *, num_tasks: int = 1, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        if num_tasks < 1:
            raise ValueError(
                "`num_tasks` value should be greater than and equal to 1, but received {num_tasks}. "
            )
        self.num_tasks = num_tasks
        for name in ("weighted_input_sum", "weighted_target_sum"):
            self._add_state(name, torch.zeros(num_tasks, dtype=torch.float64, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(
        self, input: torch.Tensor, target: torch.Tensor, weight: Union[float, int, torch.Tensor] = 1.0
    ) -> "WeightedCalibration":
        wi, wt = _weighted_calibration_update(input, target, weight, num_tasks=self.num_tasks)
        self.weighted_input_sum += wi
        self.weighted_target_sum += wt
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if torch.any(self.weighted_target_sum == 0.0):
            return torch.empty(0)
        return self.weighted_input_sum / self.weighted_target_sum

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["WeightedCalibration"]) -> "WeightedCalibration":
        for metric in metrics:
            self.weighted_input_sum += metric.weighted_input_sum.to(self.device)
            self.weighted_target_sum += metric.weighted_target_sum.to(self.device)
        return self
