"""Contiguous per-metric state buffers and the one-collective state sync.

A metric whose states are all ``sum`` / ``max`` / ``min`` tensors (counters, per-class
vectors, confusion matrices, covariance sums) keeps them as views into ONE device buffer:

    [ reduce groups | gather region: small groups ... | error-flag slot ]

* every (op, dtype) group is contiguous, so a group is one RCCL operand;
* groups larger than ``SMALL_STATE_BYTES`` ("reduce groups", e.g. a 4 MB confusion matrix)
  are all-reduced from a snapshot copy (O(|state|) bytes per rank);
* everything else - the small groups and the metric's device error flag - is the "gather
  region": ONE ``all_gather_into_tensor`` of its raw bytes, then ONE fused kernel
  (``_C.seg_reduce_rows``, csrc/kernels/sync_reduce.hip) reduces every segment over the
  ranks in rank order, so every rank ends with bit-identical states.

``sync_and_compute(MulticlassAccuracy)`` is therefore one collective on the live buffer (no
packing ``cat``, no per-state loops: the plan is cached on the buffer) plus, at ws > 1, one
reduction launch.

Groups that take the engine's own RCCL communicators (``parallel/rccl_direct.py``: 1-rank
groups by default, multi-rank groups only when opted in with ``TORCHEVAL_AMD_DIRECT_RCCL=1``)
sync with ONE grouped out-of-place all-reduce plan instead; its float sums follow RCCL's
reduction order, so for multi-rank groups the rank-ordered bit-identical guarantee above holds
on the torch.distributed path, which ``config.deterministic`` always selects.  Update kernels keep writing the same views (the K1 fast path passes
``num_correct`` / ``num_total`` pointers into the buffer).

The buffer is built lazily (first sync or reset of an eligible metric).  Any rebinding of a
state attribute (``load_state_dict``, ``to()``, a metric that assigns instead of updating in
place) is detected by a data-pointer check before each use and the buffer is rebuilt, so the
layout is an optimisation only, never a correctness assumption.

Replaces reference torcheval/metrics/toolkit.py:371-391 (``all_gather_object`` of the whole
pickled metric, then ``merge_state`` on every rank).
"""

import copy
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from torcheval_amd.parallel import collectives, rccl_direct
from torcheval_amd.parallel.distributed import backend_of

# Groups up to this size (summed over the gather region) ride the single all-gather.
SMALL_STATE_BYTES = 64 << 10
_ALIGN = 16
_FLAG_BYTES = 32  # [8] int32 slot for the metric's device error flag (<= 7 words)

_DT_CODE = {
    torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3, torch.int64: 4,
    torch.int32: 5, torch.uint8: 6, torch.bool: 7, torch.int8: 8, torch.int16: 9,
}
_OP_CODE = {"sum": 0, "max": 1, "min": 2}
_RCCL_OP = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


def _pad(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _esize(dtype: torch.dtype) -> int:
    return torch.empty((), dtype=dtype).element_size()


class _Group:
    """One (op, dtype) run of states inside the buffer."""

    __slots__ = ("op", "dtype", "off", "nbytes", "members")

    def __init__(self, op: str, dtype: torch.dtype) -> None:
        self.op = op
        self.dtype = dtype
        self.off = 0
        self.nbytes = 0
        self.members: List[Tuple[str, Tuple[int, ...], int, int]] = []  # name, shape, byte off, numel


def _flag_words(metric) -> Optional[int]:
    """Words of the metric's device error flag slot: 0 = no flag, None = not representable."""
    if not hasattr(metric, "_err"):
        return 0
    words = getattr(metric, "_err_words", None)
    if words == 0:
        return 0
    if not isinstance(words, int) or words < 0 or words >= _FLAG_BYTES // 4:
        return None
    if getattr(metric, "_err_merge", "max") != "max":
        return None
    return words


def _eligible_states(metric) -> Optional[List[Tuple[str, str, torch.Tensor]]]:
    kinds = metric._state_merge_kinds()
    if not kinds:
        return None
    out = []
    dev = None
    for name, kind in kinds.items():
        if kind not in _OP_CODE:
            return None
        v = getattr(metric, name, None)
        if not isinstance(v, torch.Tensor) or v.dtype not in _DT_CODE or v.is_sparse:
            return None
        if dev is None:
            dev = v.device
        elif v.device != dev:
            return None
        out.append((name, kind, v))
    return out


class StateBuffer:
    """The contiguous state buffer of one metric plus its cached sync plans."""

    __slots__ = ("buf", "device", "groups", "reduce_end", "gather_off", "gather_bytes", "flag_off",
                 "flag_words", "names", "ptrs", "err_obj", "default_img", "nbytes", "_seg_cache", "plans",
                 "_plain", "_props")

    # ---------------------------------------------------------------- construction
    @classmethod
    def build(cls, metric) -> Optional["StateBuffer"]:
        states = _eligible_states(metric)
        words = _flag_words(metric)
        if states is None or words is None:
            return None
        err = getattr(metric, "_err", None) if words else None
        dev = states[0][2].device
        if err is not None and (not isinstance(err, torch.Tensor) or err.dtype != torch.int32
                                or err.numel() != words or err.device != dev):
            return None
        self = cls.__new__(cls)
        self.device = dev
        groups: Dict[Tuple[str, torch.dtype], _Group] = {}
        for name, kind, v in states:
            g = groups.get((kind, v.dtype))
            if g is None:
                g = groups[(kind, v.dtype)] = _Group(kind, v.dtype)
            g.members.append((name, tuple(v.shape), g.nbytes, v.numel()))
            g.nbytes += v.numel() * v.element_size()
        # the smallest groups go to the gather region while they fit the budget
        ordered = sorted(groups.values(), key=lambda g: (g.nbytes, g.op, str(g.dtype)))
        budget, small, large = 0, [], []
        for g in ordered:
            if budget + g.nbytes <= SMALL_STATE_BYTES:
                small.append(g)
                budget += g.nbytes
            else:
                large.append(g)
        off = 0
        for g in large:
            g.off = off
            off += _pad(g.nbytes)
        self.reduce_end = off
        self.gather_off = off
        for g in small:
            g.off = off
            off += _pad(g.nbytes)
        self.flag_words = words
        self.flag_off = off if words else -1
        if words:
            off += _FLAG_BYTES
        self.gather_bytes = off - self.gather_off
        self.nbytes = off
        self.groups = large + small
        with torch.inference_mode(False):
            self.buf = torch.zeros(max(self.nbytes, _ALIGN), dtype=torch.uint8, device=dev)
            views = self.views(self.buf)
            for name, _, v in states:
                views[name].copy_(v)
            self.default_img = self._default_image(metric, states)
        for name, _, _ in states:
            setattr(metric, name, views[name])
        self.names = tuple(n for n, _, _ in states)
        if words and err is not None:
            slot = self.flag_view(self.buf)
            slot.copy_(err)
            metric._err = slot
        self.err_obj = getattr(metric, "_err", None) if words else None
        self.ptrs = tuple(getattr(metric, n).data_ptr() for n in self.names)
        # the validity check: plain attributes by object identity straight from the instance
        # dict (no data_ptr calls), properties (e.g. states with a deferred fold) through getattr
        cls = type(metric)
        self._plain = tuple((n, metric.__dict__.get(n)) for n in self.names
                            if not isinstance(getattr(cls, n, None), property) and n in metric.__dict__)
        plain = {n for n, _ in self._plain}
        self._props = tuple((n, p) for n, p in zip(self.names, self.ptrs) if n not in plain)
        self._seg_cache = None
        self.plans = {}
        metric._tea_sb = self
        return self

    def _default_image(self, metric, states) -> Optional[torch.Tensor]:
        """The state region holding every state's default (one copy resets the metric)."""
        defaults = metric._state_name_to_default
        img = torch.zeros(max(self.flag_off if self.flag_words else self.nbytes, _ALIGN),
                          dtype=torch.uint8, device=self.device)
        views = self.views(img)
        for name, _, v in states:
            d = defaults.get(name)
            if not isinstance(d, torch.Tensor) or d.dtype != v.dtype or tuple(d.shape) != tuple(v.shape):
                return None  # lazily shaped states (MSE / R2): reset() takes the generic path
            views[name].copy_(d)
        return img

    @staticmethod
    def _dead() -> "StateBuffer":
        self = StateBuffer.__new__(StateBuffer)
        self.buf = None
        return self

    def __reduce__(self):
        # pickled / deep-copied metrics rebuild their buffer on first use
        return (StateBuffer._dead, ())

    def __deepcopy__(self, memo):
        return StateBuffer._dead()

    # ---------------------------------------------------------------- layout views
    def views(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for g in self.groups:
            for name, shape, boff, n in g.members:
                o = g.off + boff
                out[name] = buf[o : o + n * _esize(g.dtype)].view(g.dtype).view(shape)
        return out

    def flag_view(self, buf: torch.Tensor) -> torch.Tensor:
        return buf[self.flag_off : self.flag_off + 4 * self.flag_words].view(torch.int32)

    def valid(self, metric) -> bool:
        if self.buf is None:
            return False
        d = metric.__dict__
        if self.flag_words and d.get("_err", getattr(metric, "_err", None)) is not self.err_obj:
            return False
        for n, obj in self._plain:
            if d.get(n) is not obj:
                return False
        try:
            for n, p in self._props:
                if getattr(metric, n).data_ptr() != p:
                    return False
        except AttributeError:
            return False
        return True

    def segments(self, base: int = 0) -> Tuple[List[int], List[int], List[int], List[int]]:
        """(byte offsets relative to the gather region + base, counts, dtype codes, op codes)."""
        if self._seg_cache is None:
            offs, counts, dts, ops = [], [], [], []
            for g in self.groups:
                if g.off < self.gather_off:
                    continue
                offs.append(g.off - self.gather_off)
                counts.append(g.nbytes // _esize(g.dtype))
                dts.append(_DT_CODE[g.dtype])
                ops.append(_OP_CODE[g.op])
            if self.flag_words:
                offs.append(self.flag_off - self.gather_off)
                counts.append(self.flag_words)
                dts.append(_DT_CODE[torch.int32])
                ops.append(_OP_CODE["max"])
            self._seg_cache = (offs, counts, dts, ops)
        offs, counts, dts, ops = self._seg_cache
        return [o + base for o in offs], counts, dts, ops

    # ---------------------------------------------------------------- reset
    def reset(self) -> bool:
        """Restore every state's default with ONE copy (views and kernel pointers kept)."""
        if self.default_img is None:
            return False
        self.buf[: self.default_img.numel()].copy_(self.default_img)
        return True


def buffer_of(metric, build: bool = True) -> Optional[StateBuffer]:
    """The metric's valid state buffer (rebuilt if a state was rebound), or None if the
    metric's states cannot live in one (cat / untyped states, variable-size error flags)."""
    sb = getattr(metric, "_tea_sb", None)
    if sb is not None and sb.valid(metric):
        return sb
    if not build:
        return None
    metric._prepare_for_merge_state()
    return StateBuffer.build(metric)


# -------------------------------------------------------------------- reductions
def _reduce_rows_torch(rows: torch.Tensor, out: torch.Tensor, segs, ws: int) -> None:
    """ATen form of the fused kernel (CPU / gloo path): one reduction per segment."""
    offs, counts, dts, ops = segs
    inv = {v: k for k, v in _DT_CODE.items()}
    for o, n, d, op in zip(offs, counts, dts, ops):
        dtype = inv[d]
        nb = n * _esize(dtype)
        seg = rows[:, o : o + nb].view(dtype)
        if dtype == torch.bool:
            red = seg.amin(0) if op == 2 else seg.amax(0)
        elif op == 0:
            red = seg.sum(0, dtype=dtype)
        else:
            red = seg.amax(0) if op == 1 else seg.amin(0)
        out[o : o + nb].view(dtype).copy_(red)


def _reduce_gathered(rows: torch.Tensor, segs, ws: int, row_bytes: int) -> torch.Tensor:
    out = torch.empty(row_bytes, dtype=torch.uint8, device=rows.device)
    if rows.is_cuda and len(segs[0]) <= 32:
        from torcheval_amd.ops import native

        native().seg_reduce_rows(rows.reshape(-1), out, ws, *segs)
    else:
        _reduce_rows_torch(rows.view(ws, row_bytes), out, segs, ws)
    return out


def _all_reduce_group(t: torch.Tensor, op: str, group, comm: Optional[int] = None) -> None:
    if t.dtype == torch.bool:  # logical or / and through uint8 max / min
        t = t.view(torch.uint8)
        op = "min" if op == "min" else "max"
    if comm is not None:  # direct RCCL on the current stream (parallel/rccl_direct.py)
        rccl_direct.all_reduce(comm, t, op)
        return
    work = dist.all_reduce(t, op=_RCCL_OP[op], group=group, async_op=collectives._issue_async(True))
    if work is not None:
        collectives._wait(work)


# -------------------------------------------------------------------- the sync
class _Plan:
    """Everything a single-metric sync needs, resolved once per (buffer, group, world size):
    the send view, the receive size, the segment table and where each state lands."""

    __slots__ = ("group", "pg", "ws", "nccl", "src", "row_bytes", "segs", "assign", "flag", "large", "fused",
                 "rank", "flag_src", "comm", "single", "gen", "rplan", "dassign", "dnames")

    def __init__(self, sb: StateBuffer, group, ws: int, metric) -> None:
        from torch.distributed.distributed_c10d import _get_default_group

        self.group = group  # held: keeps id(group) from being reused while the plan lives
        self.pg = group if group is not None else _get_default_group()
        self.ws = ws
        self.nccl = backend_of(group) == "nccl"
        self.src = sb.buf[sb.gather_off : sb.gather_off + sb.gather_bytes] if sb.gather_bytes else None
        self.row_bytes = sb.gather_bytes
        self.segs = sb.segments(0)
        self.large = [(g.off, g.nbytes, g.dtype, g.op) for g in sb.groups if g.off < sb.reduce_end]
        # (name, from the reduce snapshot?, dtype, element offset, numel, shape or None for 0-dim,
        # set through the class's property?): states are indexed out of ONE typed view per
        # (source, dtype)
        self.assign = []
        cls = type(metric)
        for g in sb.groups:
            big = g.off < sb.reduce_end
            es = _esize(g.dtype)
            for name, shape, boff, n in g.members:
                o = (g.off if big else g.off - sb.gather_off) + boff
                prop = isinstance(getattr(cls, name, None), property)
                self.assign.append((name, big, g.dtype, o // es, n, shape if shape else None, prop))
        self.flag = (sb.flag_off - sb.gather_off, 4 * sb.flag_words) if sb.flag_words else None
        # ONE collective for "one large f32 sum group + a device error flag" (confusion matrices,
        # binned counts): the flag rides the all-reduce as exact f32 (hi16, lo16) pairs in this
        # rank's slot of a [ws][words][2] block (csrc/kernels/sync_reduce.hip), so the separate
        # flag all-gather disappears; one tiny kernel merges the slots afterwards.
        small = [g for g in sb.groups if g.off >= sb.reduce_end]
        self.fused = (
            self.nccl and sb.device.type == "cuda" and sb.flag_words > 0 and not small and len(self.large) == 1
            and self.large[0][0] == 0 and self.large[0][2] == torch.float32 and self.large[0][3] == "sum"
        )
        self.rank = dist.get_rank(group) if self.fused else 0
        self.flag_src = sb.flag_view(sb.buf) if self.fused else None
        # RCCL without torch.distributed's per-call host cost (created collectively here: every
        # rank builds this plan at the same sync)
        self.comm = rccl_direct.comm_for(self.pg, ws, sb.device) if self.nccl else None
        # the whole gather region is ONE float / int SUM group and no flag (MulticlassAccuracy's
        # counters): one out-of-place all_reduce replaces all_gather + the seg_reduce launch
        gath = [g for g in sb.groups if g.off >= sb.gather_off]
        self.single = None
        if (self.comm is not None and not sb.flag_words and len(gath) == 1 and gath[0].off == sb.gather_off
                and gath[0].op == "sum" and gath[0].dtype != torch.bool):
            self.single = (gath[0].dtype, gath[0].nbytes)
        self.gen = rccl_direct.GENERATION[0]
        # the direct plan: every group (and the error flag, max-merged as int32) all-reduced OUT OF
        # PLACE from the live buffer into a result buffer of the same layout, as ONE RCCL group
        # (csrc/runtime/rccl_direct.cpp) - no snapshot copy, no gather + seg_reduce pass.  int16
        # has no RCCL type: such metrics keep the gather path.
        self.rplan = None
        self.dassign = None
        spec = direct_plan_spec(sb, cls) if self.comm is not None else None
        if spec is not None:
            ops, self.dassign = spec
            # the synced states are built as views of the result buffer inside the same native
            # call (rccl_plan_sync): one pybind round trip instead of a Python view per state;
            # plans are interned by spec, so rebuilt buffers of one layout share one native plan
            self.rplan = rccl_direct.plan_create(ops, view_specs(self.dassign))
            self.dnames = [(name, prop) for name, _, _, _, _, prop in self.dassign]


def direct_plan_spec(sb: StateBuffer, cls) -> Optional[Tuple[list, list]]:
    """The direct-RCCL plan of a buffer layout: (collective ops, state assignments), or None
    when a group has no RCCL type (int16).  Ops are ``(kind 0, src_off, dst_off, count, dtype
    code, op code)``: every group and the error flag (int32 max) all-reduced from the live
    buffer into the same offsets of a result buffer.  Assignments are ``(name, dtype, element
    offset, numel, shape or None, is_property)``."""
    if any(g.dtype == torch.int16 for g in sb.groups):
        return None
    ops = []
    for g in sb.groups:
        op = g.op if g.dtype != torch.bool else ("min" if g.op == "min" else "max")  # or / and
        ops.append((0, g.off, g.off, g.nbytes // _esize(g.dtype), _DT_CODE[g.dtype], _OP_CODE[op]))
    if sb.flag_words:
        ops.append((0, sb.flag_off, sb.flag_off, sb.flag_words, _DT_CODE[torch.int32], _OP_CODE["max"]))
    assign = []
    for g in sb.groups:
        es = _esize(g.dtype)
        for name, shape, boff, n in g.members:
            prop = isinstance(getattr(cls, name, None), property)
            assign.append((name, g.dtype, (g.off + boff) // es, n, shape if shape else None, prop))
    if sb.flag_words:
        assign.append(("_err", torch.int32, sb.flag_off // 4, sb.flag_words, (sb.flag_words,), False))
    return ops, assign


def view_specs(assign) -> List[List[int]]:
    """``[dtype code, element offset, *shape]`` per assignment (rccl_plan_set_views)."""
    return [[_DT_CODE[dt], eo, *(shape if shape is not None else ())] for _, dt, eo, _, shape, _ in assign]


def _plan_for(sb: StateBuffer, group, ws: int, metric) -> _Plan:
    key = (id(group), ws)
    plan = sb.plans.get(key)
    if plan is None or plan.group is not group or (plan.comm is not None and plan.gen != rccl_direct.GENERATION[0]):
        plan = sb.plans[key] = _Plan(sb, group, ws, metric)
    if plan.comm is not None and ws > 1 and not rccl_direct.teardown_on_failure():
        # a failure may be local to one rank: the group votes before every direct sync, and a
        # failed vote rebuilds (or leaves) the communicator on every rank at this same sync
        if rccl_direct.agree(plan.comm, plan.pg, ws, sb.device) != plan.comm:
            plan = sb.plans[key] = _Plan(sb, group, ws, metric)
    return plan


def _gather(plan: _Plan, src: torch.Tensor) -> torch.Tensor:
    """One all-gather of the raw gather region; RCCL: straight into one [ws * row] buffer."""
    if plan.nccl and collectives.current_sync_timeout() is None:
        out = torch.empty(plan.ws * plan.row_bytes, dtype=torch.uint8, device=src.device)
        if plan.comm is not None:
            rccl_direct.all_gather(plan.comm, src, out)
        else:
            dist.all_gather_into_tensor(out, src, group=plan.group)
        return out
    return collectives.all_gather_fixed_async(src, plan.group, plan.ws, blocking=True).wait()


def _direct(plan: _Plan) -> Optional[int]:
    """The plan's direct communicator when the sync may use it (no sync timeout requested:
    timeouts need torch.distributed's watchdog)."""
    return plan.comm if collectives.current_sync_timeout() is None else None


def _merged_copy(m, dst: torch.Tensor, dassign):
    """A shallow copy of ``m`` whose states view the synced buffer ``dst`` (same layout)."""
    r = object.__new__(type(m))  # a shallow copy (copy.copy costs ~4x this)
    d = r.__dict__
    getstate = getattr(type(m), "__getstate__", None)
    d.update(m.__dict__ if getstate is None else getstate(m))
    d["_tea_sb"] = None
    typed = {}
    for name, dtype, eo, n, shape, prop in dassign:
        t = typed.get(dtype)
        if t is None:
            t = typed[dtype] = dst.view(dtype)
        v = t[eo] if shape is None else t[eo : eo + n].view(shape)
        if prop:
            setattr(r, name, v)
        else:
            d[name] = v
    return r


def _sync_one_direct(m, sb: StateBuffer, plan: _Plan):
    """ONE grouped RCCL call from the live buffer into a fresh result buffer, stream-ordered
    after the updates, and the synced states as views of it - one native call; with a
    ``timeout=``, the host waits for it (``TimeoutError``)."""
    views = rccl_direct.plan_sync(plan.comm, plan.rplan, sb.buf, plan.ws)
    t = collectives.current_sync_timeout()
    if t is not None:
        rccl_direct.wait(plan.comm, t)
    r = object.__new__(type(m))  # a shallow copy (copy.copy costs ~4x this)
    d = r.__dict__
    getstate = getattr(type(m), "__getstate__", None)
    d.update(m.__dict__ if getstate is None else getstate(m))
    d["_tea_sb"] = None
    for (name, prop), v in zip(plan.dnames, views[1:]):
        if prop:
            setattr(r, name, v)
        else:
            d[name] = v
    return r


def _sync_one(m, sb: StateBuffer, plan: _Plan):
    if plan.rplan is not None:
        return _sync_one_direct(m, sb, plan)
    ws = plan.ws
    snap = None
    merged_err = None
    if plan.fused:
        from torcheval_amd.ops import native

        words = sb.flag_words
        snap = torch.empty(sb.reduce_end + ws * words * 8, dtype=torch.uint8, device=sb.device)
        native().snapshot_flags(sb.buf[: sb.reduce_end], snap, plan.flag_src, words, plan.rank, ws)
        _all_reduce_group(snap.view(torch.float32), "sum", plan.group, _direct(plan))
        merged_err = torch.empty(words, dtype=torch.int32, device=sb.device)
        native().merge_flag_slots(snap[sb.reduce_end :].view(torch.float32), merged_err, words, ws)
    elif plan.large:
        snap = sb.buf[: sb.reduce_end].clone()
        for off, nb, dtype, op in plan.large:
            _all_reduce_group(snap[off : off + nb].view(dtype), op, plan.group, _direct(plan))
    merged = None
    if plan.src is not None and not plan.fused:
        comm = _direct(plan)
        if plan.single is not None and comm is not None:
            dtype, nb = plan.single
            merged = torch.empty(plan.row_bytes, dtype=torch.uint8, device=sb.device)
            rccl_direct.all_reduce(comm, plan.src[:nb].view(dtype), "sum", out=merged[:nb].view(dtype))
        else:
            merged = _gather(plan, plan.src)
            if ws > 1:
                merged = _reduce_gathered(merged, plan.segs, ws, plan.row_bytes)
    r = object.__new__(type(m))  # a shallow copy (copy.copy costs ~4x this)
    d = r.__dict__
    getstate = getattr(type(m), "__getstate__", None)
    d.update(m.__dict__ if getstate is None else getstate(m))
    d["_tea_sb"] = None
    typed = {}
    for name, big, dtype, eo, n, shape, prop in plan.assign:
        key = (big, dtype)
        t = typed.get(key)
        if t is None:
            t = typed[key] = (snap if big else merged).view(dtype)
        v = t[eo] if shape is None else t[eo : eo + n].view(shape)
        if prop:
            setattr(r, name, v)
        else:
            d[name] = v
    if merged_err is not None:
        d["_err"] = merged_err
    elif plan.flag is not None:
        o, nb = plan.flag
        d["_err"] = merged[o : o + nb].view(torch.int32)
    return r


def sync_single(m, group, ws: int):
    """``sync_metric`` of one metric through its cached plan, or None when not eligible."""
    sb = m.__dict__.get("_tea_sb")
    if sb is None or not sb.valid(m):
        m._prepare_for_merge_state()
        sb = StateBuffer.build(m)
        if sb is None:
            return None
    plan = _plan_for(sb, group, ws, m)
    if plan.nccl and sb.device.type != "cuda":
        return None
    return _sync_one(m, sb, plan)


def fast_sync(metrics, group, ws: int) -> Optional[Dict[str, "object"]]:
    """Blocking sync of a collection whose metrics all keep their states in a StateBuffer.

    Returns ``{key: merged metric}`` (new shallow copies; the inputs are untouched) or None
    when some metric is not eligible (the caller then runs the generic engine).  Every rank
    must pass the same collection (same keys, types and state shapes)."""
    if len(metrics) == 1:  # sync_and_compute / get_synced_metric: the cached plan
        (key, m), = metrics.items()
        sb = buffer_of(m)
        if sb is None:
            return None
        plan = _plan_for(sb, group, ws, m)
        if plan.nccl and sb.device.type != "cuda":
            return None
        return {key: _sync_one(m, sb, plan)}
    issue = _fast_issue(metrics, group, ws, side=False)
    return None if issue is None else _fast_finish(issue)


_SIDE_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    """The sync engine's dedicated HIP stream on ``dev`` (one per device, created once)."""
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return s


class _FastIssue:
    """A fast sync between issue and finish: the snapshots, the receive buffer and (async) the
    event the side stream records after its collectives."""

    __slots__ = ("metrics", "sbs", "reduced", "gathered", "ws", "row_bytes", "done", "dev", "keep", "direct")


def _fast_issue(metrics, group, ws: int, side: bool) -> Optional[_FastIssue]:
    """Snapshot + issue the collectives of a state-buffer collection.  ``side``: the
    collectives go on the engine's side stream (direct RCCL only) after an event recorded
    on the current stream, so later updates on the compute stream overlap them."""
    sbs = []
    for m in metrics.values():
        sb = buffer_of(m)
        if sb is None:
            return None
        sbs.append(sb)
    dev = sbs[0].device
    if any(sb.device != dev for sb in sbs):
        return None
    nccl = backend_of(group) == "nccl"
    if nccl and dev.type != "cuda":
        return None
    comm = None
    if nccl and collectives.current_sync_timeout() is None:
        from torch.distributed.distributed_c10d import _get_default_group

        pg = group if group is not None else _get_default_group()
        comm = rccl_direct.agree(rccl_direct.comm_for(pg, ws, dev), pg, ws, dev)
    if side and comm is None:
        return None
    if comm is not None:
        plans = [_plan_for(sb, group, ws, m) for sb, m in zip(sbs, metrics.values())]
        if all(p.rplan is not None for p in plans):
            return _fast_issue_direct(metrics, sbs, plans, comm, ws, dev, side)

    # snapshots (the live buffers keep changing under later updates on the async path)
    reduced: List[Optional[torch.Tensor]] = [sb.buf[: sb.reduce_end].clone() if sb.reduce_end else None for sb in sbs]
    regions = [sb.buf[sb.gather_off : sb.gather_off + sb.gather_bytes] for sb in sbs if sb.gather_bytes]
    send = None
    if regions:
        if len(regions) > 1:
            send = torch.cat(regions)
        else:  # zero-copy send on the blocking path
            send = regions[0].clone() if side else regions[0]
    row_bytes = send.numel() if send is not None else 0
    gathered = torch.empty(ws * row_bytes, dtype=torch.uint8, device=dev) if (send is not None and comm is not None) else None

    def collectives_now() -> Optional[torch.Tensor]:
        # 1. large groups: all_reduce in place on the snapshots
        for sb, snap in zip(sbs, reduced):
            if snap is None:
                continue
            for g in sb.groups:
                if g.off < sb.reduce_end:
                    _all_reduce_group(snap[g.off : g.off + g.nbytes].view(g.dtype), g.op, group, comm)
        # 2. the gather regions: ONE all-gather
        if send is None:
            return None
        if comm is not None:
            rccl_direct.all_gather(comm, send, gathered)
            return gathered
        return collectives.all_gather_fixed_async(send, group, ws, blocking=True).wait()

    issue = _FastIssue()
    issue.metrics, issue.sbs, issue.reduced, issue.ws, issue.row_bytes, issue.dev = metrics, sbs, reduced, ws, row_bytes, dev
    issue.keep = send  # referenced until finish: the side stream reads it
    issue.done = None
    issue.direct = None
    if side:
        ready = torch.cuda.Event()
        ready.record()
        stream = _side_stream(dev)
        stream.wait_event(ready)
        with torch.cuda.stream(stream):
            issue.gathered = collectives_now()
        # allocated on the compute stream, used by RCCL on the side stream: a dropped future must
        # not let the caching allocator hand these blocks out while the collectives still run
        for t in [x for x in reduced if x is not None] + [send, gathered]:
            if t is not None:
                t.record_stream(stream)
        issue.done = torch.cuda.Event()
        issue.done.record(stream)
    else:
        issue.gathered = collectives_now()
    return issue


def _fast_issue_direct(metrics, sbs, plans, comm: int, ws: int, dev: torch.device, side: bool) -> _FastIssue:
    """Every metric's plan in ONE RCCL group, out of place into per-metric result buffers.  The
    async form snapshots each buffer (one copy; later updates keep writing the live ones) and
    runs the group on the engine's side stream."""
    dsts = [torch.empty(sb.buf.numel(), dtype=torch.uint8, device=dev) for sb in sbs]
    issue = _FastIssue()
    issue.metrics, issue.sbs, issue.ws, issue.dev = metrics, sbs, ws, dev
    issue.reduced, issue.gathered, issue.row_bytes, issue.keep = None, None, 0, None
    issue.direct = (dsts, plans)
    issue.done = None

    def run(srcs):
        rccl_direct.group_start()
        try:
            for p, src, dst in zip(plans, srcs, dsts):
                rccl_direct.plan_run(comm, p.rplan, src, dst, ws, grouped=True)
        finally:
            rccl_direct.group_end(comm, dev)

    if side:
        srcs = [sb.buf.clone() for sb in sbs]
        ready = torch.cuda.Event()
        ready.record()
        stream = _side_stream(dev)
        stream.wait_event(ready)
        with torch.cuda.stream(stream):
            run(srcs)
        for t in srcs + dsts:
            t.record_stream(stream)
        issue.keep = srcs
        issue.done = torch.cuda.Event()
        issue.done.record(stream)
    else:
        run([sb.buf for sb in sbs])
        t = collectives.current_sync_timeout()
        if t is not None:
            rccl_direct.wait(comm, t)
    return issue


def _fast_finish(issue: _FastIssue) -> Dict[str, "object"]:
    """The merged metrics of an issued fast sync (shallow copies viewing the merged buffers)."""
    if issue.done is not None:
        torch.cuda.current_stream(issue.dev).wait_event(issue.done)
    if issue.direct is not None:
        dsts, plans = issue.direct
        return {key: _merged_copy(m, dst, p.dassign) for (key, m), dst, p in zip(issue.metrics.items(), dsts, plans)}
    metrics, sbs, ws = issue.metrics, issue.sbs, issue.ws
    merged_small: Optional[torch.Tensor] = None
    if issue.gathered is not None:
        if ws == 1:
            merged_small = issue.gathered
        else:
            offs, counts, dts, ops = [], [], [], []
            base = 0
            for sb in sbs:
                if not sb.gather_bytes:
                    continue
                o, c, d, p = sb.segments(base)
                offs += o
                counts += c
                dts += d
                ops += p
                base += sb.gather_bytes
            merged_small = _reduce_gathered(issue.gathered, (offs, counts, dts, ops), ws, issue.row_bytes)

    # 3. the merged metrics: shallow copies whose states view the merged buffers
    out = {}
    base = 0
    for (key, m), sb, snap in zip(metrics.items(), sbs, issue.reduced):
        r = copy.copy(m)
        r._tea_sb = None
        for g in sb.groups:
            if g.off < sb.reduce_end:
                src, goff = snap, g.off
            else:
                src, goff = merged_small, base + g.off - sb.gather_off
            for name, shape, boff, n in g.members:
                o = goff + boff
                setattr(r, name, src[o : o + n * _esize(g.dtype)].view(g.dtype).view(shape))
        if sb.flag_words:
            o = base + sb.flag_off - sb.gather_off
            r._err = merged_small[o : o + 4 * sb.flag_words].view(torch.int32)
        if sb.gather_bytes:
            base += sb.gather_bytes
        out[key] = r
    return out


class FastPendingSync:
    """``PendingSync``-compatible handle of an async state-buffer sync on the side stream."""

    def __init__(self, issue: _FastIssue) -> None:
        self._issue = issue

    def finish(self) -> Dict[str, "object"]:
        return _fast_finish(self._issue)


def start_fast_sync(metrics, group, ws: int) -> Optional[FastPendingSync]:
    """Async form of :func:`fast_sync`: snapshot now, collectives on the engine's side HIP
    stream (direct RCCL), merge at ``finish()``.  None when not eligible.

    Opt-in (``TORCHEVAL_AMD_ASYNC_DIRECT_RCCL=1``): the engine's own communicator then runs on a
    second stream concurrently with whatever the process group runs (e.g. DDP's all-reduces),
    and two communicators in flight at once can deadlock if ranks issue them in different
    orders.  By default the async sync uses the general engine on torch.distributed's own
    async collectives (still overlapped with ``update()``, one communicator)."""
    if os.environ.get("TORCHEVAL_AMD_ASYNC_DIRECT_RCCL", "0") != "1":
        return None
    issue = _fast_issue(metrics, group, ws, side=True)
    return None if issue is None else FastPendingSync(issue)


def plan_summary(metric) -> Optional[dict]:
    """Layout of the metric's state buffer (for tests / docs): offsets, groups, collectives."""
    sb = buffer_of(metric)
    if sb is None:
        return None
    return {
        "bytes": sb.nbytes,
        "reduce_groups": [(g.op, str(g.dtype), g.off, g.nbytes) for g in sb.groups if g.off < sb.reduce_end],
        "gather_groups": [(g.op, str(g.dtype), g.off, g.nbytes) for g in sb.groups if g.off >= sb.reduce_end],
        "flag_words": sb.flag_words,
        "collectives": sum(1 for g in sb.groups if g.off < sb.reduce_end) + (1 if sb.gather_bytes else 0),
    }


__all__: Sequence[str] = ["StateBuffer", "buffer_of", "fast_sync", "plan_summary", "SMALL_STATE_BYTES"]
