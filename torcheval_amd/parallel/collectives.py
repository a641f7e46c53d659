"""Device-resident collectives for metric-state sync.

Replaces the reference's object-level sync (``dist.all_gather_object`` of whole pickled
``Metric`` objects, toolkit.py:371-391, and per-state gathers in synclib.py:61-213) with:

* ``allreduce_coalesced`` — additive / extremal states flattened into ONE contiguous bucket
  per (reduce-op, dtype) and reduced with RCCL ``all_reduce`` (async, all buckets in flight
  together).  On an 8x MI355X node each GPU has 7 xGMI links (~153 GB/s each); RCCL's
  multi-channel ring/direct algorithms spread a bucket over all of them, so one large bucket
  beats many small per-state collectives, which are latency bound (~10s of us each).
  ``bucket_cap_bytes`` (default 256 MiB) only bounds the temporary; with 288 GB of HBM a
  metric state essentially always fits in one bucket.
* ``packed_all_gather`` — an all-gather-v of an arbitrary nested tree of tensors and small
  Python values in exactly TWO collectives: an int64 header (byte counts) and one padded
  uint8 payload that carries a compact pickled skeleton (shapes / dtypes / Python leaves)
  followed by every tensor's bytes (16-B aligned).  Tensors never pass through pickle and
  never leave HBM under RCCL; received tensors are zero-copy views into the gathered buffer.
"""

import contextlib
import contextvars
import pickle
from datetime import timedelta
from collections import defaultdict
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from torcheval_amd.parallel.distributed import backend_of, transport_device

_ALIGN = 16
DEFAULT_BUCKET_CAP_BYTES = 256 << 20

_REDUCE_OPS = {
    "sum": dist.ReduceOp.SUM,
    "max": dist.ReduceOp.MAX,
    "min": dist.ReduceOp.MIN,
}


# ---------------------------------------------------------------------------- all-reduce

# Per-call deadline for the metric-sync collectives, set through
# ``sync_timeout`` / the toolkit's ``timeout=`` argument: the sync then waits on the host and
# raises TimeoutError at the deadline, on the direct RCCL path (parallel/rccl_direct.py) as on
# torch.distributed's.  None = no host wait: torch.distributed's watchdog, or the direct path's
# own watchdog thread, enforces the process group's timeout in the background.
_SYNC_TIMEOUT: "contextvars.ContextVar[Optional[timedelta]]" = contextvars.ContextVar(
    "torcheval_amd_sync_timeout", default=None
)


# Rehearsal switch: run the collective code paths even when the group has one rank (the
# shortcuts in class_shard / dist_auc otherwise skip them).  Lets a 1-GPU box execute every
# RCCL branch (reduce_scatter_tensor, all_to_all_single, all_gather_into_tensor) for real.
_COLLECTIVES_AT_WS1: "contextvars.ContextVar[bool]" = contextvars.ContextVar(
    "torcheval_amd_collectives_at_ws1", default=False
)


@contextlib.contextmanager
def collectives_at_world_size_1(enabled: bool = True):
    """Inside the block, single-rank groups take the same collective path as multi-rank ones."""
    token = _COLLECTIVES_AT_WS1.set(enabled)
    try:
        yield
    finally:
        _COLLECTIVES_AT_WS1.reset(token)


def skip_collectives(ws: int) -> bool:
    """True when a world of ``ws`` ranks may short-circuit its collectives."""
    return ws == 1 and not _COLLECTIVES_AT_WS1.get()


@contextlib.contextmanager
def sync_timeout(timeout: Optional[timedelta]):
    """Bound every metric-sync collective issued inside the block by ``timeout``."""
    token = _SYNC_TIMEOUT.set(timeout)
    try:
        yield
    finally:
        _SYNC_TIMEOUT.reset(token)


def current_sync_timeout() -> Optional[timedelta]:
    return _SYNC_TIMEOUT.get()


def _wait(work, timeout: Optional[timedelta] = None) -> None:
    t = timeout if timeout is not None else _SYNC_TIMEOUT.get()
    if t is None:
        work.wait()
        return
    try:
        ok = work.wait(t)
    except RuntimeError as e:
        raise TimeoutError(f"metric-state sync did not complete within {t}: {e}") from e
    if ok is False:
        raise TimeoutError(f"metric-state sync did not complete within {t}")

class AllReduceHandle:
    """In-flight bucketed all-reduce; ``wait()`` returns the reduced tensors in input order."""

    def __init__(self, pending, n: int) -> None:
        self._pending = pending
        self._n = n
        self._out: Optional[List[torch.Tensor]] = None
        self._timeout = _SYNC_TIMEOUT.get()  # deadline captured at issue time

    def wait(self) -> List[torch.Tensor]:
        if self._out is not None:
            return self._out
        out: List[Optional[torch.Tensor]] = [None] * self._n
        for work, flat, is_bool, layout in self._pending:
            if work is not None:
                _wait(work, self._timeout)
            if is_bool:
                flat = flat.to(torch.bool)
            off = 0
            for i, n, shape in layout:
                out[i] = flat[off : off + n].view(shape)
                off += n
        self._pending = []
        self._out = out  # type: ignore[assignment]
        return self._out  # type: ignore[return-value]


def allreduce_coalesced_async(
    tensors: Sequence[torch.Tensor],
    ops: Sequence[str],
    group: Optional[dist.ProcessGroup] = None,
    bucket_cap_bytes: int = DEFAULT_BUCKET_CAP_BYTES,
    *,
    blocking: bool = False,
) -> AllReduceHandle:
    """Issue the bucketed all-reduce of ``tensors`` (each with its op) without waiting.

    Tensors are grouped by (op, dtype) into flat buckets on the group's transport device;
    the packing copy snapshots the states, so callers may keep updating them meanwhile.
    """
    dev = transport_device(group) if len(tensors) else None
    groups: Dict[Tuple[str, torch.dtype], List[int]] = defaultdict(list)
    for i, (t, op) in enumerate(zip(tensors, ops)):
        if op not in _REDUCE_OPS:
            raise ValueError(f"unsupported reduce op {op}")
        groups[(op, t.dtype)].append(i)

    pending = []
    for (op, dtype), idxs in groups.items():
        buckets: List[List[int]] = []
        bucket: List[int] = []
        nbytes = 0
        for i in idxs:
            tb = tensors[i].numel() * tensors[i].element_size()
            if bucket and nbytes + tb > bucket_cap_bytes:
                buckets.append(bucket)
                bucket, nbytes = [], 0
            bucket.append(i)
            nbytes += tb
        if bucket:
            buckets.append(bucket)
        for b in buckets:
            parts = [tensors[i].detach().reshape(-1).to(dev) for i in b]
            flat = torch.cat(parts) if len(parts) > 1 else parts[0].clone()
            is_bool = flat.dtype == torch.bool
            if is_bool:  # no bool reductions in RCCL/gloo: logical or/and via uint8 max/min
                flat = flat.to(torch.uint8)
            work = dist.all_reduce(flat, op=_REDUCE_OPS[op], group=group, async_op=_issue_async(blocking))
            layout = [(i, tensors[i].numel(), tensors[i].shape) for i in b]
            pending.append((work, flat, is_bool, layout))
    return AllReduceHandle(pending, len(tensors))


def allreduce_coalesced(
    tensors: Sequence[torch.Tensor],
    ops: Sequence[str],
    group: Optional[dist.ProcessGroup] = None,
    bucket_cap_bytes: int = DEFAULT_BUCKET_CAP_BYTES,
) -> List[torch.Tensor]:
    """Blocking form of :func:`allreduce_coalesced_async` (inputs are left untouched)."""
    return allreduce_coalesced_async(tensors, ops, group, bucket_cap_bytes, blocking=True).wait()


# ---------------------------------------------------------------------------- all-gather-v
class _TRef:
    """Placeholder for a tensor inside a pickled skeleton."""

    __slots__ = ("offset", "nbytes", "dtype", "shape")

    def __init__(self, offset: int, nbytes: int, dtype: torch.dtype, shape: Tuple[int, ...]):
        self.offset = offset
        self.nbytes = nbytes
        self.dtype = dtype
        self.shape = shape

    def __getstate__(self):
        return (self.offset, self.nbytes, self.dtype, self.shape)

    def __setstate__(self, s):
        self.offset, self.nbytes, self.dtype, self.shape = s


class _DefaultDict:
    """Skeleton marker for a defaultdict (factory is not transported)."""

    __slots__ = ("items",)

    def __init__(self, items):
        self.items = items

    def __getstate__(self):
        return self.items

    def __setstate__(self, s):
        self.items = s


def _flatten(obj: Any, tensors: List[torch.Tensor], cursor: List[int]) -> Any:
    if isinstance(obj, torch.Tensor):
        t = obj.detach()
        if not t.is_contiguous():
            t = t.contiguous()
        nbytes = t.numel() * t.element_size()
        ref = _TRef(cursor[0], nbytes, t.dtype, tuple(t.shape))
        cursor[0] += (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        tensors.append(t)
        return ref
    if isinstance(obj, defaultdict):
        return _DefaultDict([(k, _flatten(v, tensors, cursor)) for k, v in obj.items()])
    if isinstance(obj, dict):
        return {k: _flatten(v, tensors, cursor) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_flatten(v, tensors, cursor) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_flatten(v, tensors, cursor) for v in obj)
    return obj


def _unflatten(obj: Any, buf: torch.Tensor, base: int, default_factory) -> Any:
    if isinstance(obj, _TRef):
        raw = buf[base + obj.offset : base + obj.offset + obj.nbytes]
        if obj.dtype == torch.uint8:
            return raw.view(obj.shape)
        return raw.view(obj.dtype).view(obj.shape)
    if isinstance(obj, _DefaultDict):
        return defaultdict(
            default_factory, {k: _unflatten(v, buf, base, default_factory) for k, v in obj.items}
        )
    if isinstance(obj, dict):
        return {k: _unflatten(v, buf, base, default_factory) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_unflatten(v, buf, base, default_factory) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_unflatten(v, buf, base, default_factory) for v in obj)
    return obj


def _as_bytes(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    t = t.to(dev)
    if t.dtype == torch.uint8:
        return t.reshape(-1)
    if t.dtype == torch.bool:
        return t.reshape(-1).view(torch.uint8)
    return t.reshape(-1).view(torch.uint8)


def packed_all_gather(
    tree: Any,
    group: Optional[dist.ProcessGroup] = None,
    world_size: Optional[int] = None,
    default_factory=None,
) -> List[Any]:
    """All-gather an arbitrary nested structure from every rank of ``group``.

    Returns one tree per rank (rank order).  Tensor leaves come back as views on the group's
    transport device (HBM under RCCL); Python leaves are restored verbatim.  Two collectives
    total, one host sync (to size the receive buffer).
    """
    ws = world_size if world_size is not None else dist.get_world_size(group)
    dev = transport_device(group)
    tensors: List[torch.Tensor] = []
    cursor = [0]
    skeleton = _flatten(tree, tensors, cursor)
    payload_bytes = cursor[0]
    manifest = pickle.dumps(skeleton, protocol=pickle.HIGHEST_PROTOCOL)
    mlen = len(manifest)
    mpad = (mlen + _ALIGN - 1) // _ALIGN * _ALIGN

    # header exchange: (manifest bytes, padded manifest bytes, payload bytes)
    header = torch.tensor([mlen, mpad, payload_bytes], dtype=torch.int64, device=dev)
    headers = _all_gather_fixed(header, group, ws)
    hdr = headers.view(ws, 3).cpu().tolist()
    max_total = max(h[1] + h[2] for h in hdr)
    max_total = max(max_total, _ALIGN)

    pieces: List[torch.Tensor] = []
    mtensor = torch.frombuffer(bytearray(manifest), dtype=torch.uint8)
    pieces.append(mtensor.to(dev, non_blocking=False))
    used = mlen
    if mpad > mlen:
        pieces.append(torch.zeros(mpad - mlen, dtype=torch.uint8, device=dev))
        used = mpad
    for t in tensors:
        b = _as_bytes(t, dev)
        pieces.append(b)
        n = b.numel()
        padn = (n + _ALIGN - 1) // _ALIGN * _ALIGN - n
        used += n
        if padn:
            pieces.append(torch.zeros(padn, dtype=torch.uint8, device=dev))
            used += padn
    if used < max_total:
        pieces.append(torch.zeros(max_total - used, dtype=torch.uint8, device=dev))
    send = torch.cat(pieces) if len(pieces) > 1 else pieces[0]

    recv = _all_gather_fixed(send, group, ws).view(ws, max_total)

    # one D2H copy for every rank's manifest
    max_mlen = max(h[0] for h in hdr)
    mbytes = recv[:, :max_mlen].cpu().numpy() if max_mlen > 0 else None
    out = []
    for r in range(ws):
        skel = pickle.loads(mbytes[r, : hdr[r][0]].tobytes())
        out.append(_unflatten(skel, recv[r], hdr[r][1], default_factory))
    return out


class GatherHandle:
    """In-flight fixed-size all-gather; ``wait()`` returns the flat [ws * n] result."""

    def __init__(self, work, out: Optional[torch.Tensor], outs: Optional[List[torch.Tensor]]) -> None:
        self._work = work
        self._out = out
        self._outs = outs
        self._timeout = _SYNC_TIMEOUT.get()

    def wait(self) -> torch.Tensor:
        if self._work is not None or self._outs is not None:
            if self._work is not None:
                _wait(self._work, self._timeout)
            self._work = None
            if self._outs is not None:
                self._out = torch.cat(self._outs)
                self._outs = None
        return self._out  # type: ignore[return-value]


def _issue_async(blocking: bool) -> bool:
    """Blocking callers without a deadline issue plain (stream-ordered) collectives: a Work
    handle plus ``wait()`` costs ~20 us of host time per call on RCCL (1-rank probe,
    benchmarks/rccl_primitive_latency.py)."""
    return not blocking or _SYNC_TIMEOUT.get() is not None


def all_gather_fixed_async(t: torch.Tensor, group, ws: int, *, blocking: bool = False) -> GatherHandle:
    """Issue an all-gather of equal-size 1-D tensors (one flat RCCL all-gather on HBM)."""
    t = t.reshape(-1)
    a = _issue_async(blocking)
    if backend_of(group) == "nccl":
        out = torch.empty(ws * t.numel(), dtype=t.dtype, device=t.device)
        return GatherHandle(dist.all_gather_into_tensor(out, t, group=group, async_op=a), out, None)
    outs = [torch.empty_like(t) for _ in range(ws)]
    return GatherHandle(dist.all_gather(outs, t, group=group, async_op=a), None, outs)


def _all_gather_fixed(t: torch.Tensor, group, ws: int) -> torch.Tensor:
    """All-gather equal-size 1-D tensors into one flat [ws * n] tensor."""
    return all_gather_fixed_async(t, group, ws, blocking=True).wait()


def all_gather_tensors(
    tensor: torch.Tensor, group: Optional[dist.ProcessGroup] = None
) -> List[torch.Tensor]:
    """All-gather a tensor whose shape may differ per rank (torchtnt-compatible semantics).

    Results are returned on ``tensor``'s device.
    """
    gathered = packed_all_gather(tensor, group)
    return [g.to(tensor.device) for g in gathered]
