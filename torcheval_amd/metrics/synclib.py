"""Tensor-level state sync (API parity with torcheval/metrics/synclib.py:32-291).

``sync_states(states, devices, metrics_traversal_order, process_group)`` returns, for every
rank, the nested ``{metric_name: {state_name: value}}`` dict of that rank's states.  The
reference issues several collectives per state (shape exchange + padded all-gather per
tensor, per list element, an ``all_gather_object`` per list length / int / float, plus a
``broadcast_object_list`` when some rank's list is empty).  Here the whole nested collection
goes through ONE packed all-gather-v (two collectives in total, tensors device-resident under
RCCL).  Empty lists on some ranks need no dtype/shape negotiation: every rank's list arrives
with its own length.  Fixes reference synclib.py:237 (world size taken from
``process_group``, not the default group).
"""

from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from torcheval_amd.metrics.metric import TState, _ZeroTensor
from torcheval_amd.parallel.collectives import packed_all_gather


def metrics_traversal_order(state_dict: Dict[str, Dict[str, TState]]) -> List[Tuple[str, str]]:
    """Deterministic ``(metric_name, state_name)`` order: both keys sorted."""
    order = []
    for outer_key in sorted(state_dict.keys()):
        for inner_key in sorted(state_dict[outer_key].keys()):
            order.append((outer_key, inner_key))
    return order


def sync_states(
    states: Dict[str, Dict[str, Any]],
    devices: Dict[str, torch.device],
    metrics_traversal_order: List[Tuple[str, str]],
    process_group: Optional[dist.ProcessGroup] = None,
) -> List[Dict[str, Dict[str, Any]]]:
    """Retrieve metric states from all ranks (list indexed by rank)."""
    payload: Dict[str, Dict[str, Any]] = {}
    for metric_name, state_name in metrics_traversal_order:
        value = states[metric_name][state_name]
        if not isinstance(value, (torch.Tensor, list, dict, int, float)):
            raise RuntimeError(
                f"Do not know how to sync state of type: {type(value)} for state {metric_name} {state_name}"
            )
        payload.setdefault(metric_name, {})[state_name] = value

    world_size = dist.get_world_size(process_group)
    gathered = packed_all_gather(
        payload, process_group, world_size, default_factory=_ZeroTensor(torch.device("cpu"))
    )
    out: List[Dict[str, Dict[str, Any]]] = []
    for rank_states in gathered:
        per_rank: Dict[str, Dict[str, Any]] = {}
        for metric_name, state_name in metrics_traversal_order:
            value = rank_states[metric_name][state_name]
            device = devices[metric_name]
            if isinstance(value, torch.Tensor):
                value = value.to(device).clone()
            elif isinstance(value, list):
                value = [t.to(device).clone() for t in value]
            elif isinstance(value, dict):
                value = {k: t.to(device).clone() for k, t in value.items()}
            per_rank.setdefault(metric_name, {})[state_name] = value
        out.append(per_rank)
    return out
