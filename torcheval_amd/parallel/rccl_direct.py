"""Direct RCCL communicators for the state-buffer sync (csrc/runtime/rccl_direct.cpp).

``torch.distributed``'s collectives cost ~12 us of host time per call on MI355X (Work
objects, stream-sync events, watchdog bookkeeping: ``profiles/rccl_primitive_latency_r3.json``),
which is most of a small-state ``sync_and_compute``.  For its hot path the sync engine
(``parallel/state_buffer.py``) keeps one RCCL communicator per process group of its own:
rank 0 draws an ``ncclUniqueId``, the group broadcasts it once through torch.distributed, and
each metric's sync is then ONE grouped RCCL call (a registered *plan*: every state run of the
metric's contiguous buffer all-reduced out of place into a result buffer) enqueued straight
onto the caller's current HIP stream.

Failure semantics match c10d's (reference ``toolkit.py:388`` runs under the process group's
timeout):

* every collective records a completion event that a native watchdog thread polls, with
  ``ncclCommGetAsyncError``; the deadline defaults to the process group's own timeout;
* a collective still pending at its deadline, or an async RCCL error, aborts the communicator
  (``ncclCommAbort``) and - like c10d's default async error handling - tears the process down
  with a message (``TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING=0``: keep the process; the next
  sync raises and rebuilds the communicator);
* a sync given an explicit ``timeout=`` waits for its own completion on the host and raises
  ``TimeoutError`` at the deadline; the communicator is aborted in the background and the next
  sync on the group builds a fresh one.

Bootstrapping is collective: every rank of the group reaches ``comm_for`` at the same sync
(the engine's plans are built at the same call on every rank).

Policy (``TORCHEVAL_AMD_DIRECT_RCCL``): ``auto`` (the default) uses the direct communicators
only for 1-rank groups (the forced multi-rank engine of the tests and benchmarks), because no
multi-GPU run has validated the multi-rank bootstrap yet; multi-rank groups keep
torch.distributed's collectives and the rank-ordered gather + ``seg_reduce`` path.  ``1`` opts
every group in (except under ``config.deterministic``, which keeps the rank-ordered float
sums), ``0`` keeps every collective on torch.distributed.

Agreement: with ``TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING=0`` (no teardown on a failure) a
communicator can fail on one rank only (its watchdog fired, its peers' collectives completed).
Rebuilding on that rank's own view would pair its ``broadcast`` of a new id with its peers'
next direct collective and hang, so in that mode every direct sync of a multi-rank group first
votes on the group's health (one MIN all-reduce over torch.distributed): if any rank's
communicator failed, EVERY rank drops it at the same sync and the group builds a fresh one (or
falls back to torch.distributed, again by a collective vote).  With teardown on (the default)
a failure ends the process, as c10d's does, so no rank can continue alone.
"""

import atexit
import os
from datetime import timedelta
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

_COMMS: Dict[int, tuple] = {}  # id(group) -> (group, world size, handle)
# bumped whenever a communicator is dropped: cached sync plans holding an older handle rebuild
GENERATION = [0]
_ABORTING: List[int] = []  # failed handles whose background abort a new communicator waits for
_OPS = {"sum": 0, "max": 1, "min": 2}
_DEFAULT_TIMEOUT = timedelta(minutes=10)  # c10d's NCCL default when the group reports none
# devices whose groups may get a direct communicator (tests/test_rccl_decisions.py adds "cpu" to
# drive the decision logic over gloo ranks with a fake native layer)
_DEVICE_TYPES = ("cuda",)


def enabled(ws: int = 1) -> bool:
    """Whether a group of ``ws`` ranks uses the direct communicators (see the module docstring).

    ``torcheval_amd.config.deterministic`` keeps multi-rank groups on the rank-ordered gather +
    ``seg_reduce`` path even when opted in: a direct plan all-reduces float sums in RCCL's
    order, which can differ in the last bits from the reference's sequential ``merge_state``.
    Like every collective setting, the flag must be the same on all ranks."""
    mode = os.environ.get("TORCHEVAL_AMD_DIRECT_RCCL", "auto")
    if mode == "0" or (mode != "1" and ws > 1):
        return False
    if ws > 1:
        from torcheval_amd.config import config

        if config.deterministic:
            return False
    from torcheval_amd.ops import native, native_loaded

    return native_loaded() and bool(native().rccl_available())


def teardown_on_failure() -> bool:
    """c10d-style async error handling (the default): a failed communicator ends the process."""
    return os.environ.get("TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING", "1") != "0"


def agree(handle: Optional[int], group, ws: int, device: torch.device) -> Optional[int]:
    """The handle to use for this sync of a multi-rank group, decided by ALL ranks together
    when a failure can be local (no teardown): a MIN vote of every rank's communicator health.
    A failed vote drops the communicator on every rank (``forget``) and rebuilds it collectively
    (``comm_for``), so every rank enqueues the sync on the same path.  Returns the (possibly new)
    handle or None (torch.distributed)."""
    if handle is None or ws <= 1 or teardown_on_failure():
        return handle
    if _vote(state(handle) == 0, group, device):
        return handle
    forget(handle, abort=True)
    return comm_for(group, ws, device)


def group_timeout(group, device: torch.device) -> timedelta:
    """The process group's own collective timeout (the direct path's default deadline)."""
    try:
        t = group._get_backend(device).options._timeout
        if isinstance(t, timedelta) and t.total_seconds() > 0:
            return t
    except Exception:  # noqa: BLE001 - backends without options (fake / custom groups)
        pass
    t = getattr(dist.distributed_c10d, "default_pg_nccl_timeout", None)
    return t if isinstance(t, timedelta) else _DEFAULT_TIMEOUT


def _ms(t: timedelta) -> int:
    return max(1, int(t.total_seconds() * 1000))


def comm_for(group, ws: int, device: torch.device) -> Optional[int]:
    """The direct communicator of ``group`` (created on first use, collectively), or None.

    A communicator that failed (deadline or async error) is replaced by a fresh one here, after
    its background abort has finished."""
    if device.type not in _DEVICE_TYPES or not enabled(ws):
        return None
    from torcheval_amd.ops import native

    hit = _COMMS.get(id(group))
    if hit is not None and hit[0] is group and hit[1] == ws:
        h = hit[2]
        if h is None or native().rccl_comm_state(h) == 0:
            return h
        native().rccl_wait_aborted(h, 60_000)
        del _COMMS[id(group)]
        GENERATION[0] += 1

    while _ABORTING:  # never bootstrap next to a communicator that is still being torn down
        native().rccl_wait_aborted(_ABORTING.pop(), 60_000)
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
        handle: Optional[int] = int(native().rccl_comm_init(
            uid, ws, rank, device.index if device.index is not None else 0, _ms(group_timeout(group, device))))
    except RuntimeError:
        handle = None
    if ws > 1:
        # every rank must take the same path (a rank-dependent choice would pair a direct
        # collective with a torch.distributed one and hang), so each step is voted on by the
        # whole group: first every rank must hold a communicator - the self-check is itself a
        # collective on it, which a rank without one would never join - then every rank's
        # self-check must pass.  Any failed vote sends the whole group to torch.distributed.
        if not _vote(handle is not None, group, device) or not _vote(_self_check(handle, ws, rank, device), group,
                                                                    device):
            if handle is not None:
                native().rccl_comm_destroy(handle)
            handle = None
    _COMMS[id(group)] = (group, ws, handle)
    return handle


def _vote(ok: bool, group, device: torch.device) -> bool:
    """True iff ``ok`` holds on every rank of ``group`` (one MIN all-reduce)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item()) == 1


def _self_check(handle: int, ws: int, rank: int, device: torch.device) -> bool:
    """One-time bootstrap check of a new multi-rank communicator: an out-of-place all-reduce
    and an all-gather whose results every rank can predict.  A communicator that does not
    reproduce them (a rank bound to the wrong device, a mismatched rank order) is dropped and
    the group stays on torch.distributed - the caller's MIN vote makes that choice collective."""
    from torcheval_amd.ops import native

    try:
        send = torch.tensor([rank + 1, ws - rank], dtype=torch.int32, device=device)
        red = torch.empty_like(send)
        native().rccl_all_reduce(handle, send, _OPS["sum"], red)
        gat = torch.empty(ws, dtype=torch.int32, device=device)
        native().rccl_all_gather(handle, send[:1], gat)
        want = ws * (ws + 1) // 2
        ok = red.tolist() == [want, want] and gat.tolist() == list(range(1, ws + 1))
    except RuntimeError:
        return False
    if not ok:
        import warnings

        warnings.warn(f"torcheval_amd: the direct RCCL communicator failed its bootstrap check on rank {rank} "
                      "(all-reduce / all-gather results differ); syncs use torch.distributed", stacklevel=3)
    return ok


def forget(handle: int, abort: bool = False) -> None:
    """Drop a communicator from the cache (the next ``comm_for`` rebuilds).  ``abort``: also
    abort it if it is still healthy here (a peer's failed: its collectives may never complete)."""
    for k, (_, _, h) in list(_COMMS.items()):
        if h == handle:
            del _COMMS[k]
    if abort and state(handle) == 0:
        from torcheval_amd.ops import native

        native().rccl_comm_abort(handle)
    _ABORTING.append(handle)
    GENERATION[0] += 1


def state(handle: int) -> int:
    """0 ok, 1 failed (abort pending), 2 aborted, 3 destroyed."""
    from torcheval_amd.ops import native

    return int(native().rccl_comm_state(handle))


def wait(handle: int, timeout: timedelta) -> None:
    """Block until the newest collective of ``handle`` completes; ``TimeoutError`` at the deadline
    (the communicator is then aborted in the background and replaced at the next sync)."""
    from torcheval_amd.ops import native

    if not native().rccl_wait(handle, _ms(timeout)):
        reason = native().rccl_comm_reason(handle)
        forget(handle)
        raise TimeoutError(f"metric-state sync did not complete within {timeout} ({reason})")


def plan_create(ops: Sequence[Sequence[int]], views: Sequence[Sequence[int]] = ()) -> int:
    """Register a sync plan: ``[kind, src_off, dst_off, count, dtype_code, op_code]`` per operand
    (kind 0 all-reduce of ``count`` elements, 1 all-gather of ``count`` bytes; byte offsets) and
    its synced-state views (``plan_set_views``).  Identical specs share one plan id (interned)."""
    from torcheval_amd.ops import native

    return int(native().rccl_plan_create([list(map(int, o)) for o in ops], [list(map(int, v)) for v in views]))


def plan_set_views(plan: int, views: Sequence[Sequence[int]]) -> None:
    """Register the synced-state views of a plan: ``[dtype_code, elem_off, *shape]`` each."""
    from torcheval_amd.ops import native

    native().rccl_plan_set_views(plan, [list(map(int, v)) for v in views])


def plan_sync(handle: int, plan: int, src: torch.Tensor, ws: int) -> List[torch.Tensor]:
    """Fresh result buffer + the plan's grouped collectives + the state views: [result, *views]."""
    from torcheval_amd.ops import native

    try:
        return native().rccl_plan_sync(handle, plan, src, ws)
    except RuntimeError:
        if state(handle) != 0:  # failed earlier (watchdog): rebuild at the next sync
            forget(handle)
        raise


def plan_run(handle: int, plan: int, src: torch.Tensor, dst: torch.Tensor, ws: int, grouped: bool = False) -> None:
    from torcheval_amd.ops import native

    try:
        native().rccl_plan_run(handle, plan, src, dst, ws, grouped)
    except RuntimeError:
        if state(handle) != 0:  # failed earlier (watchdog): rebuild at the next sync
            forget(handle)
        raise


def group_start() -> None:
    from torcheval_amd.ops import native

    native().rccl_group_start()


def group_end(track: int = -1, device: Optional[torch.device] = None) -> None:
    from torcheval_amd.ops import native

    native().rccl_group_end(track, device.index if device is not None and device.index is not None else 0)


def all_gather(handle: int, src: torch.Tensor, out: torch.Tensor) -> None:
    from torcheval_amd.ops import native

    native().rccl_all_gather(handle, src, out)


def all_reduce(handle: int, t: torch.Tensor, op: str, out: Optional[torch.Tensor] = None) -> None:
    """In place, or (``out``) out of place: the send buffer is left untouched."""
    from torcheval_amd.ops import native

    native().rccl_all_reduce(handle, t, _OPS[op], out)


def destroy_all() -> None:
    """Destroy every direct communicator (after its work drains) and stop the watchdog.
    Call it before ``dist.destroy_process_group()``; also registered with atexit."""
    from torcheval_amd.ops import native, native_loaded

    if not native_loaded():
        return
    handles: List[int] = [h for _, _, h in _COMMS.values() if h is not None]
    _COMMS.clear()
    for handle in handles:
        try:
            native().rccl_comm_destroy(handle)
        except RuntimeError:
            pass
    try:
        native().rccl_shutdown()
    except RuntimeError:
        pass


atexit.register(destroy_all)
