"""K5b wrappers (csrc/kernels/rowsums.hip + its host twin csrc/runtime/rowsums_host.cpp):
per-row weighted sums merged straight into metric state tensors.

``update_states(x, t, w, outs)`` computes, for each row of ``x`` ([rows, n], or any tensor
flattened to one row), the requested FP64 statistics and applies them to the given outputs
in one native call:

==========  =====================================  ==========================
stat        value per row                          typical state
==========  =====================================  ==========================
``WX``      sum w * x   (w: tensor or scalar)      Sum / Mean / CTR clicks
``WT``      sum w * t                              weighted calibration
``W``       sum w       (scalar w: w * n)          Mean weights / CTR weights
``SSE``     sum (x - t)^2                          PSNR
``WSSE``    sum w (x - t)^2                        MeanSquaredError
``WTT``     sum w t^2                              R2Score
``TMIN``    min t,  ``TMAX``: max t                PSNR auto range
``COUNT``   n                                      PSNR observations
``RANGE``   merged TMAX output - merged TMIN out   PSNR data_range
==========  =====================================  ==========================

ops: ``SET`` (=), ``ADD`` (+=), ``MIN``, ``MAX`` - each in the output's own dtype (f32/f64),
exactly like ``state = state op value``.  ROCm tensors: one kernel launch (two for rows longer
than 64K elements); CPU tensors up to ``HOST_MAX`` elements: the C++ host twin (one call
instead of 4-6 ATen dispatches); larger CPU tensors keep the ATen path.
"""

from typing import Optional, Sequence, Tuple, Union

import torch

import torcheval_amd.ops as _ops
from torcheval_amd.ops import native, native_loaded

WX, WT, W, SSE, WSSE, WTT, TMIN, TMAX, COUNT, RANGE = range(10)
SET, ADD, MIN, MAX = range(4)
FIRST_ROW = 4  # or-ed into an op: a scalar output fed by row 0 only
HOST_MAX = 1 << 13
_IN_DTYPES = (torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int64, torch.int32,
              torch.int16, torch.int8, torch.uint8, torch.bool)


def supported(x: torch.Tensor, *others: Optional[torch.Tensor], states: Sequence[torch.Tensor] = ()) -> bool:
    """Whether the fused path applies: native build present, ROCm tensors (or small CPU ones),
    supported dtypes, states f32/f64 on the inputs' device."""
    if not native_loaded():
        return False
    if x.is_cuda:
        if _ops.DISABLE_HIP:  # read at call time: A/B benchmarks toggle it
            return False
    elif x.numel() > HOST_MAX:
        return False
    if x.dtype not in _IN_DTYPES:
        return False
    for o in others:
        if o is not None and (o.dtype not in _IN_DTYPES or o.device != x.device):
            return False
    for s in states:
        if s.dtype not in (torch.float32, torch.float64) or s.device != x.device:
            return False
    return True


_STATE_DTYPES = (torch.float32, torch.float64)


def fast_ok(x: torch.Tensor, w, *states: torch.Tensor) -> bool:
    """One cheap check for the per-batch class updates: native build, ROCm tensors (or CPU ones
    of at most HOST_MAX elements), supported dtypes, a scalar or same-shape tensor weight,
    f32 / f64 states on the input's device."""
    if _ops._C is None or x.dtype not in _IN_DTYPES:
        return False
    if x.is_cuda:
        if _ops.DISABLE_HIP:
            return False
    elif x.numel() > HOST_MAX:
        return False
    dev = x.device
    if isinstance(w, torch.Tensor):
        if w.shape != x.shape or w.dtype not in _IN_DTYPES or w.device != dev:
            return False
    elif not isinstance(w, (float, int)):
        return False
    for st in states:
        if st.dtype not in _STATE_DTYPES or st.device != dev:
            return False
    return True


def weight_ok(input: torch.Tensor, weight) -> bool:
    """Weights the fused update accepts without changing the reference's error behaviour
    (anything else takes the ATen path and raises there)."""
    if isinstance(weight, torch.Tensor):
        return weight.size() == input.size()
    return isinstance(weight, (float, int))


def update_states(
    x: torch.Tensor,
    t: Optional[torch.Tensor],
    w: Union[None, float, int, torch.Tensor],
    outs: Sequence[Tuple[torch.Tensor, int, int]],
    *,
    rows: int = 1,
) -> None:
    """Apply ``(output, stat, op)`` triples for ``x`` / ``t`` / ``w`` viewed as ``[rows, n]``
    (any shape: the native side views it as rows x numel / rows)."""
    if isinstance(w, torch.Tensor):
        wt, ws = w, 1.0
    else:
        wt, ws = None, float(1.0 if w is None else w)
    update(x, t, wt, ws, [o for o, _, _ in outs], [s * 8 + op for _, s, op in outs], rows)


def update(x: torch.Tensor, t: Optional[torch.Tensor], w: Optional[torch.Tensor], w_scalar: float,
           outs: list, codes: list, rows: int = 1) -> None:
    """Lean form for the per-batch metric updates: outputs and packed codes (stat * 8 + op).
    Eager calls take the pybind entry (less host time); under torch.compile the dispatcher op
    (CPU host twin / GPU kernel, with a Meta kernel) keeps the update in the graph."""
    if _ops.compiling():
        torch.ops.torcheval_amd.row_sums(x, t, w, w_scalar, outs, codes, rows)
        return
    native().row_sums(x, t, w, w_scalar, outs, codes, rows)


def code(stat: int, op: int) -> int:
    return stat * 8 + op
