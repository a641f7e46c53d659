"""Direct RCCL communicators for the state-buffer sync (csrc/runtime/rccl_direct.cpp).

``torch.distributed``'s collectives cost ~12 us of host time per call on MI355X (Work
objects, stream-sync events, watchdog bookkeeping: ``profiles/rccl_primitive_latency_r3.json``),
which is most of a small-state ``sync_and_compute``.  For its hot path the sync engine
(``parallel/state_buffer.py``) keeps one RCCL communicator per process group of its own:
rank 0 draws an ``ncclUniqueId``, the group broadcasts it once through torch.distributed, and
``ncclAllGather`` / ``ncclAllReduce`` are then enqueued straight onto the caller's current HIP
stream (ordered after the update kernels, no cross-stream events).

Bootstrapping is collective: every rank of the group reaches ``comm_for`` at the same sync
(the engine's plans are built at the same call on every rank).  ``TORCHEVAL_AMD_DIRECT_RCCL=0``
keeps every collective on torch.distributed (e.g. when a program interleaves its own
collectives on other streams with metric syncs in a rank-dependent order).
"""

import atexit
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

_COMMS: Dict[int, tuple] = {}  # id(group) -> (group, world size, handle)
_OPS = {"sum": 0, "max": 1, "min": 2}


def enabled() -> bool:
    if os.environ.get("TORCHEVAL_AMD_DIRECT_RCCL", "1") == "0":
        return False
    from torcheval_amd.ops import native, native_loaded

    return native_loaded() and bool(native().rccl_available())


def comm_for(group, ws: int, device: torch.device) -> Optional[int]:
    """The direct communicator of ``group`` (created on first use, collectively), or None."""
    if device.type != "cuda" or not enabled():
        return None
    hit = _COMMS.get(id(group))
    if hit is not None and hit[0] is group and hit[1] == ws:
        return hit[2]
    from torcheval_amd.ops import native

    rank = dist.get_rank(group)
    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        native().rccl_unique_id(uid)
    if ws > 1:  # the group's own backend carries the 128-byte id once
        dev_uid = uid.to(device)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(dev_uid, src=src, group=group)
        uid = dev_uid.cpu()
    try:
        handle: Optional[int] = int(native().rccl_comm_init(uid, ws, rank, device.index if device.index is not None else 0))
    except RuntimeError:
        handle = None
    if ws > 1:
        # every rank must take the same path: one failed init sends the whole group back to
        # torch.distributed (a rank-dependent choice would pair a direct collective with a
        # torch.distributed one and hang)
        ok = torch.tensor([1 if handle is not None else 0], dtype=torch.int32, device=device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if int(ok.item()) == 0 and handle is not None:
            native().rccl_comm_destroy(handle)
            handle = None
    _COMMS[id(group)] = (group, ws, handle)
    return handle


def all_gather(handle: int, src: torch.Tensor, out: torch.Tensor) -> None:
    from torcheval_amd.ops import native

    native().rccl_all_gather(handle, src, out)


def all_reduce(handle: int, t: torch.Tensor, op: str, out: Optional[torch.Tensor] = None) -> None:
    """In place, or (``out``) out of place: the send buffer is left untouched."""
    from torcheval_amd.ops import native

    native().rccl_all_reduce(handle, t, _OPS[op], out)


def destroy_all() -> None:
    """Destroy every direct communicator (also registered with atexit)."""
    from torcheval_amd.ops import native, native_loaded

    if not native_loaded():
        return
    for _, _, handle in list(_COMMS.values()):
        if handle is None:
            continue
        try:
            native().rccl_comm_destroy(handle)
        except RuntimeError:
            pass
    _COMMS.clear()


atexit.register(destroy_all)
