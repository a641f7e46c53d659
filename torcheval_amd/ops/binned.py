"""K4 binned-histogram wrapper (csrc/kernels/binned.hip) + the equivalent ATen path.

``binned_counts(scores, target, thr, mode)`` returns float32 (tp, fp, fn) of shape [T, C] for
a [n, C] score view: tp[k, j] = #positives of column j with score >= thr[k], fp likewise for
negatives, fn = positives - tp.  ``mode`` 0: ``target`` is a [n, C] {0,1} view; mode 1:
``target`` is [n] class labels (positive when label == j).
"""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import compiling, native, use_native


def binned_counts(
    scores: torch.Tensor,
    target: torch.Tensor,
    thr: torch.Tensor,
    mode: int,
    out: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Accumulate into ``out`` ([T, C] float32 views) or return fresh counts."""
    from torcheval_amd.metrics.functional.tensor_utils import _is_uniform_linspace

    T, C = thr.numel(), scores.shape[1]
    uniform = _is_uniform_linspace(thr) and thr.dtype == torch.float32 and thr.device == scores.device
    thr = thr.to(device=scores.device)
    if out is None:
        buf = torch.zeros(3, T, C, dtype=torch.float32, device=scores.device)
        out = (buf[0], buf[1], buf[2])
    if use_native(scores) and target.is_cuda and T <= 2048:
        t = target
        if t.dtype == torch.bool:
            t = t.to(torch.uint8)
        thr32 = thr.to(torch.float32).contiguous()
        if compiling():
            torch.ops.torcheval_amd.binned_counts(scores, t, thr32, int(mode), *out, int(uniform))
        else:
            native().binned_counts(scores, t, thr32, int(mode), *out, uniform=int(uniform))
        return out
    if _cpu_binned(scores, target, thr, mode):
        # small CPU batches: one C++ call (the ATen chain below is ~10 dispatches)
        native().cpu_binned_counts(scores, target, thr, int(mode), *out)
        return out
    tp, fp, fn = _binned_counts_aten(scores, target, thr, mode)
    out[0].add_(tp)
    out[1].add_(fp)
    out[2].add_(fn)
    return out


def _cpu_binned(scores: torch.Tensor, target: torch.Tensor, thr: torch.Tensor, mode: int) -> bool:
    import torcheval_amd.ops as ops

    if ops.compiling() or scores.is_cuda or target.is_cuda or thr.is_cuda or ops.DISABLE_HIP or not ops.native_loaded():
        return False
    if scores.numel() > (1 << 16) or scores.dtype not in (torch.float32, torch.float64):
        return False
    ok_t = (torch.int64, torch.int32) if mode == 1 else (torch.int64, torch.int32, torch.bool, torch.uint8,
                                                         torch.float32, torch.float64)
    return target.dtype in ok_t and thr.dtype in (torch.float32, torch.float64)


def _binned_counts_aten(
    scores: torch.Tensor, target: torch.Tensor, thr: torch.Tensor, mode: int
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    n, C = scores.shape
    T = thr.numel()
    bins = torch.searchsorted(thr.to(scores.dtype).contiguous(), scores.contiguous(), right=True)
    if mode == 1:
        pos = (target[:, None] == torch.arange(C, device=scores.device)[None, :]).long()
    else:
        pos = (target == 1).long()
    flat = (bins * C + torch.arange(C, device=scores.device)[None, :]) * 2 + pos
    hist = torch.bincount(flat.reshape(-1), minlength=(T + 1) * C * 2).view(T + 1, C, 2).to(torch.float64)
    suffix = hist.flip(0).cumsum(0).flip(0)
    tp = suffix[1:, :, 1]
    fp = suffix[1:, :, 0]
    fn = hist[:, :, 1].sum(0)[None, :] - tp
    return tp.float(), fp.float(), fn.float()


def binned_finalize_supported(*counts: torch.Tensor) -> bool:
    return all(
        use_native(c) and c.dtype == torch.float32 and c.dim() == 2 and c.shape == counts[0].shape
        for c in counts
    )


def binned_finalize(
    tp: torch.Tensor, fp: torch.Tensor, fn: Optional[torch.Tensor] = None, *, auroc: bool = True, auprc: bool = False
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """One launch: float64 [R] binned AUROC and/or float32 [R] binned AUPRC from [T, R] counts."""
    tp, fp = tp.contiguous(), fp.contiguous()
    fn = fn.contiguous() if fn is not None else None
    rows = tp.shape[1]
    out_roc = torch.empty(rows, dtype=torch.float64, device=tp.device) if auroc else None
    out_pr = torch.empty(rows, dtype=torch.float32, device=tp.device) if auprc else None
    native().binned_finalize(tp, fp, fn, out_roc, out_pr)
    return out_roc, out_pr


def binned_curve(tp: torch.Tensor, fp: torch.Tensor, fn: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """One launch: float32 [R, T+1] precision (NaN -> 1, closed by 1) and recall (closed by 0)
    from [T, R] counts - the binned PR-curve compute chain."""
    T, rows = tp.shape
    prec = torch.empty(rows, T + 1, dtype=torch.float32, device=tp.device)
    rec = torch.empty(rows, T + 1, dtype=torch.float32, device=tp.device)
    native().binned_finalize(tp, fp, fn, None, None, prec, rec)
    return prec, rec
