"""Process-group helpers (owned replacements for the torchtnt utilities the reference uses).

The reference pulls ``PGWrapper`` / ``init_from_env`` from torchtnt (toolkit.py:22,
metric_class_tester.py:19); torchtnt is not part of this stack, so the equivalents live here.

On MI355X one process drives one GPU; the ``"nccl"`` backend of ``torch.distributed`` is RCCL,
which moves bytes over the xGMI point-to-point links.  ``transport_device`` picks where a
collective's buffers must live for the group's backend (HBM for RCCL, host for gloo).
"""

import os
from datetime import timedelta
from typing import Any, List, Optional

import torch
import torch.distributed as dist


class PGWrapper:
    """Thin wrapper that behaves sensibly when ``torch.distributed`` is not initialised."""

    def __init__(self, pg: Optional[dist.ProcessGroup] = None) -> None:
        self.pg = pg

    def get_world_size(self) -> int:
        if not dist.is_available() or not dist.is_initialized():
            return 1
        return dist.get_world_size(self.pg)

    def get_rank(self) -> int:
        if not dist.is_available() or not dist.is_initialized():
            return 0
        return dist.get_rank(self.pg)

    def barrier(self) -> None:
        if dist.is_available() and dist.is_initialized():
            if backend_of(self.pg) == "nccl":
                dist.barrier(self.pg, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(self.pg)

    def all_gather_object(self, obj_list: List[Any], obj: Any) -> None:
        if self.get_world_size() == 1:
            obj_list[0] = obj
            return
        dist.all_gather_object(obj_list, obj, group=self.pg)

    def broadcast_object_list(self, obj_list: List[Any], src: int = 0) -> None:
        if self.get_world_size() == 1:
            return
        dist.broadcast_object_list(obj_list, src=src, group=self.pg)


def get_world_size(pg: Optional[dist.ProcessGroup] = None) -> int:
    return PGWrapper(pg).get_world_size()


_WS_CACHE: dict = {}  # id(group) -> (group, world size); a group's size never changes


def cached_world_size(pg: Optional[dist.ProcessGroup] = None) -> int:
    """``PGWrapper(pg).get_world_size()`` with the per-group size cached (the sync hot path:
    torch's lookup walks the group registry on every call, ~3 us)."""
    if not dist.is_available() or not dist.is_initialized():
        return 1
    g = pg if pg is not None else dist.group.WORLD
    hit = _WS_CACHE.get(id(g))
    if hit is not None and hit[0] is g:
        return hit[1]
    ws = dist.get_world_size(g)
    _WS_CACHE[id(g)] = (g, ws)  # holds the group: its id cannot be reused while cached
    return ws


def get_rank(pg: Optional[dist.ProcessGroup] = None) -> int:
    return PGWrapper(pg).get_rank()


def backend_of(pg: Optional[dist.ProcessGroup] = None) -> str:
    backend = dist.get_backend(pg)
    return str(backend).lower()


def transport_device(pg: Optional[dist.ProcessGroup] = None) -> torch.device:
    """Device the group's collectives operate on: current HIP device for RCCL, else CPU."""
    if backend_of(pg) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def get_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_from_env(
    *,
    device_type: Optional[str] = None,
    pg_backend: Optional[str] = None,
    pg_timeout: timedelta = timedelta(minutes=30),
) -> torch.device:
    """Initialise the default process group from torchrun-style env vars; return the device.

    One process per GPU: ``LOCAL_RANK`` selects the HIP device and the backend defaults to
    ``"nccl"`` (RCCL over xGMI) when the device is a GPU, ``"gloo"`` on CPU.
    """
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        device = torch.device("cuda", get_local_rank())
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size > 1 and dist.is_available() and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = pg_backend or ("nccl" if device_type == "cuda" else "gloo")
        kwargs = {}
        if backend == "nccl":
            kwargs["device_id"] = device
        dist.init_process_group(backend=backend, timeout=pg_timeout, **kwargs)
    return device
