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
"""

import copy
from collections import defaultdict
from typing import Any, Dict, List, MutableMapping, Optional

import torch
import torch.distributed as dist

from torcheval_amd.metrics.metric import Metric, _ZeroTensor
from torcheval_amd.parallel import collectives

_PLAIN = (int, float, str, bool, type(None))
_SKIP_ATTRS = {"_state_name_to_default", "_state_merge_kind", "_device"}


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


def sync_metric_collection(
    metrics: MutableMapping[str, Metric],
    process_group: Optional[dist.ProcessGroup] = None,
    world_size: Optional[int] = None,
) -> Dict[str, Metric]:
    """Return a dict of new metrics whose states are merged over every rank of the group."""
    group = process_group
    ws = world_size if world_size is not None else dist.get_world_size(group)

    for m in metrics.values():
        m._prepare_for_merge_state()

    reduce_tensors: List[torch.Tensor] = []
    reduce_ops: List[str] = []
    reduce_slots: List[tuple] = []  # (key, state_name)
    gather_tree: Dict[str, Any] = {}
    typed: Dict[str, bool] = {}

    for key, m in metrics.items():
        is_typed = _is_typed(m)
        typed[key] = is_typed
        kinds = m._state_merge_kinds()
        if is_typed:
            cat_states = {}
            for name, kind in kinds.items():
                value = getattr(m, name)
                if kind in ("sum", "max", "min"):
                    reduce_tensors.append(value)
                    reduce_ops.append(kind)
                    reduce_slots.append((key, name))
                else:
                    cat_states[name] = list(value)
            if cat_states:
                gather_tree[key] = {"states": cat_states}
        else:
            states = {name: getattr(m, name) for name in kinds}
            extras = {
                k: v
                for k, v in vars(m).items()
                if k not in kinds and k not in _SKIP_ATTRS and _is_plain(v)
            }
            gather_tree[key] = {"states": states, "extras": extras}

    # issue the all-reduce buckets first (async), then the all-gather-v
    reduced = collectives.allreduce_coalesced_async(reduce_tensors, reduce_ops, group)
    gathered = (
        collectives.packed_all_gather(
            gather_tree, group, ws, default_factory=_ZeroTensor(torch.device("cpu"))
        )
        if gather_tree
        else None
    )
    reduced_values = reduced.wait()

    result: Dict[str, Metric] = {}
    # typed metrics: clone + fill reduced / concatenated states
    for key, m in metrics.items():
        if not typed[key]:
            continue
        out = _shallow_clone(m)
        result[key] = out
        if gathered is not None and key in gather_tree:
            for name in gather_tree[key]["states"]:
                merged: List[torch.Tensor] = []
                for r in range(ws):
                    merged.extend(t.to(m.device) for t in gathered[r][key]["states"][name])
                setattr(out, name, merged)
    for (key, name), value in zip(reduce_slots, reduced_values):
        m = metrics[key]
        setattr(result[key], name, value.to(m.device))

    # untyped metrics: shadow per rank + the metric's own merge_state (reference semantics)
    for key, m in metrics.items():
        if typed[key]:
            continue
        shadows = []
        for r in range(ws):
            sh = _shallow_clone(m)
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
    return result


def sync_metric(
    metric: Metric,
    process_group: Optional[dist.ProcessGroup] = None,
    world_size: Optional[int] = None,
) -> Metric:
    return sync_metric_collection({"_": metric}, process_group, world_size)["_"]
