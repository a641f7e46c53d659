"""RetrievalPrecision class metric (parity: metrics/ranking/retrieval_precision.py:23-199).

The reference keeps, per query, a Python list entry of top-k scores / targets and updates
them in a loop over queries (``i in indexes`` is one host sync per query, then cat + topk +
gather per query); compute loops again with a ``1 in target`` host check per query.

Here the state is dense and device-resident, and neither update nor compute synchronises:

* ``k`` given: ``topk`` / ``target`` are ``[num_queries, k]`` (score-descending, padded with
  -inf / 0) plus ``count`` (valid entries per query, <= k).  On ROCm (f32 state, k <= 64,
  num_queries <= 8192) one update is the K10b kernel chain (csrc/kernels/retrieval.hip):
  per-query histogram, scan, a scatter of the batch into per-query segments, and one wave
  per query selecting the top-k of old row + segment - 4 launches, no sort.  Otherwise: one
  composite-key sort of the batch by (query, score desc) - a single int64 radix sort -
  segment starts from an index_add histogram, a gather of every query's best k batch items,
  and one row-wise ``topk`` of [num_queries, 2k] candidates (old top-k + batch top-k).
* ``k=None`` (every item is retrieved): the top-"all" is the whole history, so the state is the
  per-query sums it reduces to - ``relevant`` (sum of targets), ``positives`` (count of
  target == 1) and ``items`` - merged with ``merge="sum"`` (one RCCL all-reduce when synced).

Samples whose query index is outside [0, num_queries) are ignored, as in the reference.
``load_state_dict`` also accepts the reference's list-of-tensors state dicts.
"""

from typing import Any, Dict, Iterable, Optional, Union

import torch
from typing_extensions import Literal

from torcheval_amd.metrics.functional.ranking import (
    _retrieval_precision_param_check,
    _retrieval_precision_update_input_check,
)
from torcheval_amd.metrics.metric import Metric, inference_update

__all__ = ["RetrievalPrecision"]

_NEG_INF = float("-inf")


def _desc_key_f32(x: torch.Tensor) -> torch.Tensor:
    """int64 in [0, 2^32): ascending order of the key = descending order of the f32 scores
    (NaN first, as torch.topk ranks it)."""
    b = x.contiguous().view(torch.int32).to(torch.int64)
    u = torch.where(b >= 0, b + (1 << 31), -1 - b)  # ascending float order, unsigned
    return (1 << 32) - 1 - u


class RetrievalPrecision(Metric[torch.Tensor]):
    """
    Precision@k per query with a bounded-memory, device-resident streaming top-k.

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
        Q = num_queries
        if k is not None:
            self._add_state("topk", torch.full((Q, k), _NEG_INF, device=self.device))
            self._add_state("target", torch.zeros(Q, k, device=self.device))
            self._add_state("count", torch.zeros(Q, dtype=torch.int64, device=self.device))
        else:
            for name in ("relevant", "positives", "items"):
                self._add_state(name, torch.zeros(Q, dtype=torch.float64, device=self.device), merge="sum")

    # ------------------------------------------------------------------ update
    @inference_update
    def update(
        self, input: torch.Tensor, target: torch.Tensor, indexes: Optional[torch.Tensor] = None
    ) -> "RetrievalPrecision":
        _retrieval_precision_update_input_check(input, target, num_queries=self.num_queries, indexes=indexes)
        Q = self.num_queries
        if Q > 1 and indexes is None:
            raise ValueError("`indexes` must be passed during update() when num_queries > 1.")
        dev = self._state_device()
        if self.k is not None and self._native_topk(input, target, indexes):
            return self
        input, target = input.to(dev), target.to(dev)
        if Q == 1:
            q = torch.zeros(input.shape[0], dtype=torch.int64, device=dev)
        else:
            q = indexes.to(dev).to(torch.int64)
            q = torch.where((q >= 0) & (q < Q), q, torch.full_like(q, Q))  # ignored -> dump row Q
        if self.k is None:
            self._update_sums(input, target, q)
        else:
            self._update_topk(input, target, q)
        return self

    def _state_device(self) -> torch.device:
        return (self.topk if self.k is not None else self.relevant).device

    def _update_sums(self, input: torch.Tensor, target: torch.Tensor, q: torch.Tensor) -> None:
        Q = self.num_queries
        t = target.to(torch.float64)
        stats = torch.zeros(3, Q + 1, dtype=torch.float64, device=q.device)
        stats[0].index_add_(0, q, t)
        stats[1].index_add_(0, q, (target == 1).to(torch.float64))
        stats[2].index_add_(0, q, torch.ones_like(t))
        self.relevant += stats[0, :Q]
        self.positives += stats[1, :Q]
        self.items += stats[2, :Q]

    def _native_topk(self, input: torch.Tensor, target: torch.Tensor, indexes: Optional[torch.Tensor]) -> bool:
        """K10b path: f32 state on ROCm, 1 <= k <= 64, num_queries <= 8192."""
        from torcheval_amd.ops import native, use_native

        if not (use_native(input) and self.topk.is_cuda and self.topk.dtype == torch.float32
                and self.target.dtype == torch.float32 and 1 <= self.k <= 64 and self.num_queries <= 8192
                and input.dtype in (torch.float32, torch.float16, torch.bfloat16)
                and input.shape[0] < 2**31
                and target.dtype in (torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.uint8, torch.bool)):
            return False
        x = input.to(self.topk.device, torch.float32).contiguous()
        t = target.to(self.topk.device, torch.float32).contiguous()
        q = None
        if self.num_queries > 1:
            q = indexes.to(self.topk.device, torch.int64).contiguous()
        self.topk, self.target, self.count = self.topk.contiguous(), self.target.contiguous(), self.count.contiguous()
        native().retrieval_topk_update(x, t, q, self.topk, self.target, self.count)
        return True

    def _update_topk(self, input: torch.Tensor, target: torch.Tensor, q: torch.Tensor) -> None:
        Q, k, n = self.num_queries, self.k, input.shape[0]
        dev = q.device
        vdt = torch.promote_types(self.topk.dtype, input.dtype)
        tdt = torch.promote_types(self.target.dtype, target.dtype)
        # batch order: query ascending, score descending (one int64 sort for f32 scores)
        if input.dtype == torch.float32:
            perm = torch.sort(q * (1 << 32) + _desc_key_f32(input)).indices
        else:
            by_score = torch.sort(input, descending=True, stable=True).indices
            perm = by_score[torch.sort(q[by_score], stable=True).indices]
        counts = torch.zeros(Q + 1, dtype=torch.int64, device=dev).index_add_(0, q, torch.ones_like(q))
        starts = counts.cumsum(0) - counts
        j = torch.arange(k, device=dev)
        take = j[None, :] < counts[:Q, None]                      # [Q, k]: the query's best k
        pos = torch.where(take, starts[:Q, None] + j[None, :], torch.zeros_like(j)[None, :])
        src = perm[pos.clamp(max=max(n - 1, 0))] if n else pos
        bv = torch.where(take, input.to(vdt)[src], torch.full((), _NEG_INF, dtype=vdt, device=dev)) if n \
            else torch.full((Q, k), _NEG_INF, dtype=vdt, device=dev)
        bt = torch.where(take, target.to(tdt)[src], torch.zeros((), dtype=tdt, device=dev)) if n \
            else torch.zeros(Q, k, dtype=tdt, device=dev)
        cand_v = torch.cat([self.topk.to(vdt), bv], 1)
        cand_t = torch.cat([self.target.to(tdt), bt], 1)
        self.topk, sel = cand_v.topk(k, dim=1)
        self.target = cand_t.gather(1, sel)
        self.count = torch.clamp(self.count + counts[:Q], max=k)

    # ------------------------------------------------------------------ compute
    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if self.k is None:
            nb, has_pos, n_items = self.relevant, self.positives > 0, self.items
            total = n_items
        else:
            valid = torch.arange(self.k, device=self.count.device)[None, :] < self.count[:, None]
            tgt = torch.where(valid, self.target, torch.zeros_like(self.target))
            nb = tgt.sum(1)
            has_pos = ((tgt == 1) & valid).any(1)
            n_items = self.count
            total = torch.clamp(self.count, max=self.k) if self.limit_k_to_size else torch.full_like(self.count, self.k)
        rp = (nb / total).to(torch.float32)
        if self.empty_target_action == "err":
            bad = (n_items > 0) & ~has_pos
            if bool(bad.any()):  # raising needs the host: only this mode reads back
                i = int(bad.nonzero()[0, 0])
                raise ValueError(f"no positive value found in target={self._query_targets(i)}.")
            empty_val = float("nan")
        else:
            empty_val = {"pos": 1.0, "neg": 0.0, "skip": float("nan")}.get(self.empty_target_action, float("nan"))
        rp = torch.where(has_pos, rp, torch.full_like(rp, empty_val))
        rp = torch.where(n_items > 0, rp, torch.full_like(rp, float("nan")))
        rp = rp.to(self.device)
        return rp.nanmean() if self.avg == "macro" else rp

    def _query_targets(self, i: int) -> torch.Tensor:
        if self.k is None:
            return torch.zeros(int(self.items[i]))
        return self.target[i, : int(self.count[i])].float()

    # ------------------------------------------------------------------ merge / checkpoint
    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["RetrievalPrecision"]) -> "RetrievalPrecision":
        metrics = list(metrics)
        if self.k is None:
            for m in metrics:
                self.relevant += m.relevant.to(self.relevant.device)
                self.positives += m.positives.to(self.positives.device)
                self.items += m.items.to(self.items.device)
            return self
        dev = self.topk.device
        vals = torch.cat([self.topk] + [m.topk.to(dev) for m in metrics], 1)
        tgts = torch.cat([self.target] + [m.target.to(dev) for m in metrics], 1)
        self.topk, sel = vals.topk(self.k, dim=1)  # top-k of the union = global top-k
        self.target = tgts.gather(1, sel)
        total = self.count + sum(m.count.to(dev) for m in metrics)
        self.count = torch.clamp(total, max=self.k)
        return self

    def load_state_dict(self, state_dict: Dict[str, Any], strict: bool = True) -> None:
        """Also accepts the reference's state dicts (``topk`` / ``target`` lists per query)."""
        sd = dict(state_dict)
        if isinstance(sd.get("topk"), list) or isinstance(sd.get("target"), list):
            topk_l, tgt_l = sd.pop("topk", []), sd.pop("target", [])
            fresh = RetrievalPrecision(k=self.k, limit_k_to_size=self.limit_k_to_size, num_queries=self.num_queries,
                                       empty_target_action=self.empty_target_action, avg=self.avg, device=self.device)
            for i, (v, t) in enumerate(zip(topk_l, tgt_l)):
                if v.numel():
                    fresh.update(v.reshape(-1), t.reshape(-1), torch.full((v.numel(),), i, dtype=torch.int64))
            sd.update(fresh.state_dict())
        super().load_state_dict(sd, strict)
