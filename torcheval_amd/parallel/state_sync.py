"""Typed metric-state synchronisation engine (the L4 sync layer, MI355X-native).

Reference behaviour (toolkit.py:206-260, 371-391): every rank pickles its whole ``Metric``
(states, hyper-parameters, any ``nn.Module``), ``all_gather_object``s it, and every rank
computes ``clone(gathered[0]).to(device).merge_state(gathered[1:])``.  The result is the
same object on every rank.

Here the same result is produced with device-resident RCCL traffic:

* **typed metrics** — every state declares a merge kind (``Metric._add_state(merge=...)``):
  ``sum``/``max``/``min`` tensors of every metric in the collection are packed into one
  bucket per (op, dtype) and ``all_reduce``d (O(|state|) bytes per rank instead of the
  reference's O(world_size * |state|)); ``cat`` list states are all-gathered (v) and
  concatenated in rank order.  ``merge_state`` is not called.
* **untyped metrics** (any state with merge kind ``None``, custom user metrics) — every state
  plus the small per-rank Python attributes travel through ONE packed all-gather-v and the
  metric's own ``merge_state`` runs on rank-ordered shadows, reproducing the reference result
  exactly (including order-dependent merges such as window metrics).

The all-reduce buckets are issued before the all-gather, so both are in flight together.
``start_sync_collection`` / ``PendingSync.finish`` split the exchange so the all-reduce can
overlap further ``update()`` calls (``toolkit.sync_and_compute_async``).
"""

import copy
from collections import defaultdict
from typing import Any, Dict, List, MutableMapping, Optional

import torch
import torch.distributed as dist

from torcheval_amd.metrics.metric import Metric, _ZeroTensor
from torcheval_amd.parallel import collectives
from torcheval_amd.parallel.distributed import transport_device

_PLAIN = (int, float, str, bool, type(None))
_SKIP_ATTRS = {"_state_name_to_default", "_state_merge_kind", "_device"}
# Device error flags (``_err``: int32 vectors of <= 6 words written by the native kernels'
# input validation) travel in one fixed [M, 8] int32 all-gather; word 7 carries the length.
_ERR_SLOT = 8


def _has_err_flag(metric: Metric) -> bool:
    return hasattr(metric, "_err")


def _pack_err_flags(metrics, keys: List[str], dev: torch.device) -> torch.Tensor:
    packed = torch.zeros(len(keys), _ERR_SLOT, dtype=torch.int32, device=dev)
    for i, key in enumerate(keys):
        e = getattr(metrics[key], "_err", None)
        if isinstance(e, torch.Tensor) and e.numel():
            n = min(e.numel(), _ERR_SLOT - 1)
            packed[i, :n] = e.reshape(-1)[:n].to(device=dev, dtype=torch.int32)
            packed[i, _ERR_SLOT - 1] = n
    return packed.reshape(-1)


def _merge_err_flags(flat: torch.Tensor, ws: int, keys: List[str], metrics, result) -> None:
    """Every rank adopts the error record of the lowest rank that flagged one (so all ranks
    raise the same error in ``compute()``); each synced metric gets its own flag tensor."""
    g = flat.view(ws, len(keys), _ERR_SLOT)
    first = (g[:, :, 0] != 0).to(torch.int32).argmax(0)  # lowest flagged rank (0 if none)
    chosen = g[first, torch.arange(len(keys), device=g.device)]  # [M, 8]
    for i, key in enumerate(keys):
        local = getattr(metrics[key], "_err", None)
        if isinstance(local, torch.Tensor):
            n, dev = local.numel(), local.device
        else:  # this rank never ran a flagged update: size the flag from the record itself
            n = int(chosen[i, _ERR_SLOT - 1].item())
            if n == 0:
                continue
            dev = metrics[key].device
        result[key]._err = chosen[i, :n].to(dev).clone()


def _is_plain(v: Any) -> bool:
    if isinstance(v, _PLAIN):
        return True
    if isinstance(v, tuple):
        return all(_is_plain(x) for x in v)
    return False


def _is_typed(metric: Metric) -> bool:
    kinds = metric._state_merge_kinds()
    if not kinds:
        return False
    for name, kind in kinds.items():
        value = getattr(metric, name)
        if kind is None:
            return False
        if kind in ("sum", "max", "min") and not isinstance(value, torch.Tensor):
            return False
        if kind == "cat" and not isinstance(value, list):
            return False
    return True


def _shallow_clone(metric: Metric) -> Metric:
    return copy.copy(metric)


class PendingSync:
    """An in-flight metric sync (see :func:`start_sync_collection`).

    At creation every state that will travel has been snapshotted (the all-reduce buckets are
    packing copies already queued on RCCL's own stream; gathered states are cloned), so the
    caller may keep calling ``update()`` on the original metrics while the all-reduce runs.
    ``finish()`` issues the all-gather-v (if any), waits, and assembles the merged metrics.
    """

    def __init__(self, metrics, group, ws, typed, gather_tree, reduced, reduce_slots, outs,
                 err_keys=(), err_gather=None) -> None:
        self._metrics = metrics
        self._err_keys = list(err_keys)
        self._err_gather = err_gather
        self._group = group
        self._ws = ws
        self._typed = typed
        self._gather_tree = gather_tree
        self._reduced = reduced
        self._reduce_slots = reduce_slots
        self._outs = outs
        self._result: Optional[Dict[str, Metric]] = None

    def finish(self) -> Dict[str, Metric]:
        if self._result is not None:
            return self._result
        metrics, ws, gather_tree = self._metrics, self._ws, self._gather_tree
        gathered = (
            collectives.packed_all_gather(
                gather_tree, self._group, ws, default_factory=_ZeroTensor(torch.device("cpu"))
            )
            if gather_tree
            else None
        )
        reduced_values = self._reduced.wait()

        result: Dict[str, Metric] = {}
        # typed metrics: clone + fill reduced / concatenated states
        for key, m in metrics.items():
            if not self._typed[key]:
                continue
            out = self._outs[key]
            result[key] = out
            if gathered is not None and key in gather_tree:
                for name in gather_tree[key]["states"]:
                    merged: List[torch.Tensor] = []
                    for r in range(ws):
                        merged.extend(t.to(m.device) for t in gathered[r][key]["states"][name])
                    setattr(out, name, merged)
        for (key, name), value in zip(self._reduce_slots, reduced_values):
            setattr(result[key], name, value.to(metrics[key].device))

        # untyped metrics: shadow per rank + the metric's own merge_state (reference semantics)
        for key, m in metrics.items():
            if self._typed[key]:
                continue
            shadows = []
            for r in range(ws):
                sh = _shallow_clone(self._outs[key])
                entry = gathered[r][key]
                for attr, v in entry["extras"].items():
                    setattr(sh, attr, v)
                for name, v in entry["states"].items():
                    if isinstance(v, dict):
                        v = defaultdict(_ZeroTensor(m.device), v)
                    setattr(sh, name, v)
                shadows.append(sh)
            base = shadows[0].to(m.device)
            # detach base states from the shared receive buffer before in-place merges
            for name in m._state_name_to_default:
                v = getattr(base, name)
                if isinstance(v, torch.Tensor):
                    setattr(base, name, v.clone())
                elif isinstance(v, list):
                    setattr(base, name, [t.clone() for t in v])
            result[key] = base.merge_state(shadows[1:])
        if self._err_gather is not None:
            _merge_err_flags(self._err_gather.wait(), ws, self._err_keys, metrics, result)
        self._result = result
        return result


def _snapshot(v: Any) -> Any:
    if isinstance(v, torch.Tensor):
        return v.detach().clone()
    if isinstance(v, list):
        return [_snapshot(x) for x in v]
    if isinstance(v, dict):
        return {k: _snapshot(x) for k, x in v.items()}
    return v


def start_sync_collection(
    metrics: MutableMapping[str, Metric],
    process_group: Optional[dist.ProcessGroup] = None,
    world_size: Optional[int] = None,
    *,
    snapshot: bool = True,
) -> PendingSync:
    """Snapshot the states of ``metrics`` and issue the bucketed all-reduce asynchronously.

    The all-reduce rides RCCL's internal stream, so it overlaps whatever the caller enqueues
    next on the compute stream (typically more ``update()`` calls).  With ``snapshot=False``
    gathered states are referenced instead of cloned (the blocking path, which finishes
    immediately, uses this to avoid a copy)."""
    group = process_group
    ws = world_size if world_size is not None else dist.get_world_size(group)

    for m in metrics.values():
        m._prepare_for_merge_state()

    reduce_tensors: List[torch.Tensor] = []
    reduce_ops: List[str] = []
    reduce_slots: List[tuple] = []  # (key, state_name)
    gather_tree: Dict[str, Any] = {}
    typed: Dict[str, bool] = {}
    outs: Dict[str, Metric] = {}
    keep = _snapshot if snapshot else (lambda v: v)

    for key, m in metrics.items():
        is_typed = _is_typed(m)
        typed[key] = is_typed
        kinds = m._state_merge_kinds()
        outs[key] = _shallow_clone(m)
        if is_typed:
            cat_states = {}
            for name, kind in kinds.items():
                value = getattr(m, name)
                if kind in ("sum", "max", "min"):
                    reduce_tensors.append(value)
                    reduce_ops.append(kind)
                    reduce_slots.append((key, name))
                else:
                    cat_states[name] = keep(list(value))
            if cat_states:
                gather_tree[key] = {"states": cat_states}
        else:
            states = {name: keep(getattr(m, name)) for name in kinds}
            extras = {
                k: v
                for k, v in vars(m).items()
                if k not in kinds and k not in _SKIP_ATTRS and _is_plain(v)
            }
            gather_tree[key] = {"states": states, "extras": extras}

    # the packing copies inside snapshot the reduce states; RCCL runs them asynchronously
    reduced = collectives.allreduce_coalesced_async(reduce_tensors, reduce_ops, group)
    err_keys = [key for key, m in metrics.items() if _has_err_flag(m)]
    err_gather = None
    if err_keys:  # same keys on every rank: the flag attribute exists from __init__
        flags = _pack_err_flags(metrics, err_keys, transport_device(group))
        err_gather = collectives.all_gather_fixed_async(flags, group, ws)
    return PendingSync(metrics, group, ws, typed, gather_tree, reduced, reduce_slots, outs,
                       err_keys, err_gather)


def sync_metric_collection(
    metrics: MutableMapping[str, Metric],
    process_group: Optional[dist.ProcessGroup] = None,
    world_size: Optional[int] = None,
) -> Dict[str, Metric]:
    """Return a dict of new metrics whose states are merged over every rank of the group."""
    return start_sync_collection(metrics, process_group, world_size, snapshot=False).finish()


def sync_metric(
    metric: Metric,
    process_group: Optional[dist.ProcessGroup] = None,
    world_size: Optional[int] = None,
) -> Metric:
    return sync_metric_collection({"_": metric}, process_group, world_size)["_"]
