"""K5 weighted-sums dispatch shared by the regression metrics."""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import _C, compiling, native, use_native
from torcheval_amd.ops import rowsums as _rs

# K5b statistic -> cpu_moments_update destination (sse, st, stt, sw)
_CPU_SLOT = {_rs.WSSE: 0, _rs.SSE: 0, _rs.WT: 1, _rs.WTT: 2, _rs.W: 3, _rs.COUNT: 3}


def _native(input: torch.Tensor, target: torch.Tensor, w: Optional[torch.Tensor] = None) -> bool:
    from torcheval_amd.ops.reductions import moments_supported

    return use_native(input) and moments_supported(input, target, w) and input.numel() > 0


def _update(
    input: torch.Tensor, target: torch.Tensor, sample_weight: Optional[torch.Tensor]
) -> Tuple[torch.Tensor, torch.Tensor]:
    squared_error = torch.square(target - input)
    if sample_weight is None:
        return squared_error.sum(dim=0), torch.tensor(target.size(0), device=target.device)
    if squared_error.ndim == 2:
        sample_weight = sample_weight.unsqueeze(-1)
    return (squared_error * sample_weight).sum(dim=0), sample_weight.sum(dim=0).squeeze()


def _state(metric, name: str) -> torch.Tensor:
    """A state without folding pending device sums (metrics/_pending.py), else getattr."""
    v = metric.__dict__.get("_pv_" + name)
    return v if v is not None else getattr(metric, name)


def _promote_lazy(metric, names, input: torch.Tensor):
    """The reference's lazy shape promotion of 0-d states to [d] on the first 2-D update
    (done here up front so the fused kernels can accumulate in place).  Returns the states by
    name (the promoted tensors themselves: under torch.compile a re-read of the instance dict
    can see the pre-promotion value), or None when the states and the batch disagree in shape
    (the ATen path then reproduces the reference's broadcast)."""
    d = input.shape[1] if input.ndim == 2 else 1
    states = {n: _state(metric, n) for n in names}
    if input.ndim == 2 and all(s.ndim == 0 for s in states.values()):
        for n, s in list(states.items()):
            states[n] = torch.zeros(d, dtype=s.dtype, device=s.device) + s
            setattr(metric, n, states[n])
        return states
    ok = all(s.numel() == d and s.ndim == (1 if input.ndim == 2 else 0) for s in states.values())
    return states if ok else None


def _cpu_update(metric, input: torch.Tensor, target: torch.Tensor, w: Optional[torch.Tensor], sums, scalars) -> bool:
    """Small CPU batch: one host call (csrc/runtime/cpu_metrics.cpp cpu_moments_update) adds
    the FP64 batch sums into the f32 states; it declines (False) any dtype / shape / state
    layout it does not take, so the checks stay in C++."""
    n = input.numel()
    if n == 0 or n > _rs.HOST_MAX or _C is None or compiling():
        return False
    states = _promote_lazy(metric, [s for s, _ in sums], input) if input.ndim == 2 else None
    if input.ndim == 2 and states is None:
        return False
    kw = [None, None, None, None]  # sse, st, stt, sw
    count = False
    for name, stat in sums:
        kw[_CPU_SLOT[stat]] = states[name] if states is not None else _state(metric, name)
    for name, stat in scalars:
        kw[_CPU_SLOT[stat]] = _state(metric, name)
        count = count or stat == _rs.COUNT
    return _C.cpu_moments_update(input, target, w, kw[0], kw[1], kw[2], kw[3], count)


def fused_regression_update(metric, input: torch.Tensor, target: torch.Tensor, w: Optional[torch.Tensor],
                            sums, scalars) -> bool:
    """One-call update of per-column regression sums straight into ``metric``'s f32 states.

    ``sums``: (state name, K5b stat) of the [d] states; ``scalars``: (state name, stat) of the
    0-d ones (a count or a weight total).  ROCm [n, d] batches run K5 column moments
    (coalesced over d) accumulating into the states; ROCm [n] batches and small CPU batches
    run K5b (``ops/rowsums.py``) over the transposed view; small CPU batches one host call
    (csrc/runtime/cpu_metrics.cpp cpu_moments_update).  False: take the ATen path."""
    if not input.is_cuda and _cpu_update(metric, input, target, w, sums, scalars):
        return True
    if input.dtype != torch.float32 or target.dtype != torch.float32:
        return False
    if w is not None and (w.dtype != torch.float32 or w.ndim != 1):
        return False
    names = [n for n, _ in sums] + [n for n, _ in scalars]
    if not all(_state(metric, n).dtype == torch.float32 and _state(metric, n).device == input.device for n in names):
        return False
    if input.is_cuda and input.ndim == 2:
        if not _native(input, target, w):
            return False
        states = _promote_lazy(metric, [n for n, _ in sums], input)
        if states is None:
            return False
        key = {_rs.WSSE: "sse", _rs.SSE: "sse", _rs.WT: "st", _rs.WTT: "stt", _rs.W: "sw", _rs.COUNT: "sw"}
        spec = {key[stat]: n for n, stat in list(sums) + list(scalars)}
        kw = {"sse": None, "st": None, "stt": None, "sw": None}
        for k, n in spec.items():
            kw[k] = states[n] if n in states else _state(metric, n)
        if getattr(metric, "_pend_states", ()) and not compiling():
            # deferred mode (metrics/_pending.py): the launch only adds FP64 partials to the
            # metric's pending slots; the states fold them in when read
            d = input.shape[1]
            need = sum(b for k, b in (("sse", 1), ("st", 2), ("stt", 4)) if kw[k] is not None)
            # the slot layout comes from C++ (tea_kernels.h moments_ns_of; it rejects a statistic
            # set the fold kernel cannot read)
            pend = metric._pend_buffer(native().column_moments_pend_numel(d, need), input.device, spec)
            slots = native().column_moments_pend(input, target, w, kw["sse"], kw["st"], kw["stt"], None, kw["sw"], pend)
            if slots:
                metric._pend_mark(slots, spec)
                return True
        from torcheval_amd.ops.reductions import column_moments

        column_moments(input, target, w, **kw)
        return True
    if not _rs.supported(input, target, w) or input.numel() == 0:
        return False
    if _promote_lazy(metric, [n for n, _ in sums], input) is None:
        return False
    rows = input.shape[1] if input.ndim == 2 else 1
    x2 = input.t() if input.ndim == 2 else input.reshape(1, -1)
    t2 = target.t() if target.ndim == 2 else target.reshape(1, -1)
    w2 = None if w is None else w.reshape(1, -1).expand(rows, -1)
    outs = [(getattr(metric, n).reshape(-1), stat, _rs.ADD) for n, stat in sums]
    outs += [(getattr(metric, n), stat, _rs.ADD | _rs.FIRST_ROW) for n, stat in scalars]
    _rs.update_states(x2, t2, w2, outs, rows=rows)
    return True
