"""Wrappers of the K5 / K6 fused reductions (csrc/kernels/reductions.hip)."""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import compiling, native

_FLOATISH = (torch.float32, torch.float64, torch.float16, torch.bfloat16)
_ANY = _FLOATISH + (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)


def moments_supported(*ts: Optional[torch.Tensor]) -> bool:
    return all(t is None or (t.is_cuda and t.dtype in _ANY) for t in ts)


def column_moments(
    x: Optional[torch.Tensor],
    t: Optional[torch.Tensor],
    w: Optional[torch.Tensor] = None,
    *,
    sse: Optional[torch.Tensor] = None,
    st: Optional[torch.Tensor] = None,
    stt: Optional[torch.Tensor] = None,
    sx: Optional[torch.Tensor] = None,
    sw: Optional[torch.Tensor] = None,
    overwrite: bool = False,
) -> None:
    """Accumulate (or, with ``overwrite``, write) weighted column moments of [n, d] (or [n])
    x / t into float32 outputs."""
    if x is not None and x.dim() == 1:
        x = x[:, None]
    if t is not None and t.dim() == 1:
        t = t[:, None]
    if t is not None and t.dtype == torch.bool:
        t = t.to(torch.uint8)
    if compiling():  # the dispatcher op (Meta kernel): keeps a compiled update in one graph
        torch.ops.torcheval_amd.column_moments(x, t, w, sse, st, stt, sx, sw, int(overwrite), 0, None, 0)
        return
    native().column_moments(x, t, w, sse, st, stt, sx, sw, int(overwrite))


def mse_fused(
    x: torch.Tensor, t: torch.Tensor, w: Optional[torch.Tensor], raw_values: bool
) -> torch.Tensor:
    """Functional mean_squared_error in two launches: K5 partials, then a finalize that also
    divides by the clamped signed weight total (raw values: per column; uniform average: one
    single-block fold of per-block {sse, weight} pairs, sum_j sse_j / (d sw))."""
    d = x.shape[1] if x.dim() == 2 else 1
    x2 = x[:, None] if x.dim() == 1 else x
    t2 = t[:, None] if t.dim() == 1 else t
    if t2.dtype == torch.bool:
        t2 = t2.to(torch.uint8)
    buf = torch.empty(d + 1, dtype=torch.float32, device=x.device)
    out = torch.empty(d if raw_values else (), dtype=torch.float32, device=x.device)
    _cm = torch.ops.torcheval_amd.column_moments if compiling() else native().column_moments
    _cm(x2, t2, w, buf[:d], None, None, None, buf[d:], 1, 1 if raw_values else 2, out, 0)
    if raw_values and x.dim() == 1:
        return out[0]  # [1] -> scalar, as sse.sum(dim=0) of a 1-D error is 0-d
    return out


_R2_MODES = {"raw_values": 3, "uniform_average": 4, "variance_weighted": 5}


def r2_fused(x: torch.Tensor, t: torch.Tensor, multioutput: str, num_regressors: int) -> torch.Tensor:
    """Functional r2_score: K5 partials, then a finalize that forms tss, r2 (and the adjusted
    score) per column, plus one single-block launch for the uniform / variance-weighted mean."""
    d = x.shape[1] if x.dim() == 2 else 1
    x2 = x[:, None] if x.dim() == 1 else x
    t2 = t[:, None] if t.dim() == 1 else t
    if t2.dtype == torch.bool:
        t2 = t2.to(torch.uint8)
    buf = torch.empty(3, d, dtype=torch.float32, device=x.device)
    mode = _R2_MODES[multioutput]
    out = torch.empty(d if mode == 3 else (), dtype=torch.float32, device=x.device)
    _cm = torch.ops.torcheval_amd.column_moments if compiling() else native().column_moments
    _cm(x2, t2, None, buf[0], buf[1], buf[2], None, None, 1, mode, out, int(num_regressors))
    if mode == 3 and x.dim() == 1:
        return out[0]
    return out


def ne_sums(
    input: torch.Tensor,
    target: torch.Tensor,
    weight: Optional[torch.Tensor],
    from_logits: bool,
    err: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """float64 [rows, 3] = (sum w*BCE, sum w*t, sum w) per row, and the range flag."""
    x = input if input.dim() == 2 else input[None, :]
    t = target if target.dim() == 2 else target[None, :]
    w = None if weight is None else (weight if weight.dim() == 2 else weight[None, :])
    x, t = x.contiguous(), t.contiguous()
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    if w is not None:
        w = w.contiguous()
    out = torch.zeros(x.shape[0], 3, dtype=torch.float64, device=x.device)
    flag = err if err is not None else torch.zeros(1, dtype=torch.int32, device=x.device)
    from torcheval_amd.config import config

    _ne = torch.ops.torcheval_amd.ne_sums if compiling() else native().ne_sums
    _ne(x, t, w, bool(from_logits), out, flag, bool(config.deterministic))
    return out, flag
