"""Class-dimension sharded sync (SURVEY.md §2.8 "TP analog").

The data-parallel sync (``sync_and_compute``) all-reduces every count state, so each rank ends
with the whole [C, C] confusion matrix or [T, C] binned counts and computes every class's
result.  For extreme class counts (C = 10^5 classes x T = 200 thresholds x 3 count states is
240 MB of fp32) that moves ``2 (ws-1)/ws`` of the state per rank over xGMI and repeats the
compute ws times.  Here the counts are **reduce-scattered** along the class dimension instead:

* one ``reduce_scatter_tensor`` (``(ws-1)/ws`` of the state per rank: half an all-reduce's ring
  traffic) leaves rank r with the global counts of classes ``[r*c, (r+1)*c)``;
* each rank computes only its classes;
* the per-class results (C floats) are all-gathered, or - for the confusion matrix - the row
  block stays sharded (``ShardedRows``), which is what a caller with a [10^5, 10^5] matrix wants.

Gloo has no reduce-scatter: on gloo (CPU test rehearsal) the same API all-reduces then slices, so
results are identical by construction.
"""

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F

from torcheval_amd.parallel.collectives import _wait, skip_collectives

__all__ = ["reduce_scatter_classes", "class_sharded_compute", "sharded_confusion_matrix", "ShardedRows"]


def _ws_rank(group) -> Tuple[int, int]:
    if not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _local_only(ws: int) -> bool:
    return not dist.is_initialized() or skip_collectives(ws)


def reduce_scatter_classes(
    t: torch.Tensor, *, dim: int = 0, group: Optional[dist.ProcessGroup] = None
) -> Tuple[torch.Tensor, int, int]:
    """Sum ``t`` over ranks and keep this rank's slice of dimension ``dim``.

    Returns ``(shard, start, stop)``: ``shard`` is the summed ``t.narrow(dim, start, stop-start)``
    moved to the front (shape ``[stop-start, *other dims]``).  Chunks are ``ceil(C/ws)`` classes
    (the last ranks may own fewer or none)."""
    ws, rank = _ws_rank(group)
    C = t.shape[dim]
    chunk = -(-C // ws)
    start, stop = min(rank * chunk, C), min((rank + 1) * chunk, C)
    front = t.movedim(dim, 0)
    if _local_only(ws):
        return front.contiguous(), 0, C
    rest = front.shape[1:]
    if dist.get_backend(group) == "gloo":
        full = front.contiguous().clone()
        _wait(dist.all_reduce(full, group=group, async_op=True))
        return full[start:stop].clone(), start, stop
    pad = chunk * ws - C
    buf = front.contiguous()
    if pad:
        buf = torch.cat([buf, buf.new_zeros((pad,) + tuple(rest))])
    out = buf.new_empty((chunk,) + tuple(rest))
    _wait(dist.reduce_scatter_tensor(out, buf, group=group, async_op=True))
    return out[: stop - start], start, stop


def _gather_classes(local: torch.Tensor, C: int, group) -> torch.Tensor:
    """Concatenate every rank's per-class result (chunked as in ``reduce_scatter_classes``)."""
    ws, _ = _ws_rank(group)
    if _local_only(ws):
        return local
    chunk = -(-C // ws)
    padded = local.new_zeros((chunk,) + tuple(local.shape[1:]))
    padded[: local.shape[0]] = local
    out = local.new_empty((ws * chunk,) + tuple(local.shape[1:]))
    if dist.get_backend(group) == "gloo":
        _wait(dist.all_gather(list(out.chunk(ws)), padded, group=group, async_op=True))
    else:
        _wait(dist.all_gather_into_tensor(out, padded, group=group, async_op=True))
    return out[:C]


@dataclass
class ShardedRows:
    """Rows ``[start, stop)`` of a [C, C] matrix that lives sharded across ranks."""

    rows: torch.Tensor
    start: int
    stop: int
    num_classes: int

    def gather(self, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
        """The whole [C, C] matrix on every rank (one all-gather)."""
        return _gather_classes(self.rows, self.num_classes, group)


def sharded_confusion_matrix(
    metric, *, normalize: Optional[str] = "__metric__", group: Optional[dist.ProcessGroup] = None
) -> ShardedRows:
    """Row-sharded ``compute()`` of a ``MulticlassConfusionMatrix`` (row = target class).

    ``normalize`` defaults to the metric's own; "true" normalises rows locally, "pred" and "all"
    need the column / grand totals: one extra all-reduce of C+1 floats."""
    from torcheval_amd.metrics.functional.classification.confusion_matrix import _confusion_matrix_param_check

    if normalize == "__metric__":
        normalize = metric.normalize
    C = metric.num_classes
    _confusion_matrix_param_check(C, normalize)
    metric._check_device_errors()
    rows, start, stop = reduce_scatter_classes(metric.confusion_matrix, dim=0, group=group)
    if normalize in ("pred", "all"):
        col = torch.cat([rows.abs().sum(0), rows.sum().reshape(1)]).float()
        ws, _ = _ws_rank(group)
        if not _local_only(ws):
            _wait(dist.all_reduce(col, group=group, async_op=True))
        if normalize == "pred":
            rows = rows.float() / col[:C].clamp_min(1e-12)
        else:
            rows = rows.float() / col[C]
    elif normalize == "true":
        rows = F.normalize(rows.float(), p=1, dim=1)
    return ShardedRows(rows, start, stop, C)


def class_sharded_compute(metric, *, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """``compute()`` of a class-count metric with the class dimension reduce-scattered across
    ranks (each rank reduces and finalises only its classes; C results are all-gathered).
    Same value on every rank as ``sync_and_compute(metric)``.

    Supported: ``MulticlassBinnedAUPRC``, ``MultilabelBinnedAUPRC`` ([T, C] counts) and
    ``MulticlassConfusionMatrix`` (full matrix; use ``sharded_confusion_matrix`` to keep it
    sharded)."""
    from torcheval_amd.metrics.classification.binned_auprc import MulticlassBinnedAUPRC, MultilabelBinnedAUPRC
    from torcheval_amd.metrics.classification.confusion_matrix import MulticlassConfusionMatrix
    from torcheval_amd.metrics.functional.classification.binned_auprc import _binned_riemann

    if isinstance(metric, MulticlassConfusionMatrix):
        return sharded_confusion_matrix(metric, group=group).gather(group)
    if isinstance(metric, (MulticlassBinnedAUPRC, MultilabelBinnedAUPRC)):
        # one collective for the three [T, C] states: stacked class-major [C, 3, T]
        counts = torch.stack([metric.num_tp, metric.num_fp, metric.num_fn], 0).permute(2, 0, 1)
        local, _, _ = reduce_scatter_classes(counts, dim=0, group=group)
        C = counts.shape[0]
        if local.shape[0]:
            tp, fp, fn = (local[:, i].t() for i in range(3))  # [T, c]
            part = _binned_riemann(tp.contiguous(), fp.contiguous(), fn.contiguous())
        else:
            part = torch.zeros(0, dtype=torch.float32, device=counts.device)
        auprc = _gather_classes(part, C, group)
        return auprc.mean() if metric.average == "macro" else auprc
    raise TypeError(f"class_sharded_compute does not support {type(metric).__name__}")
