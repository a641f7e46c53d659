"""Shared tie-aware ROC / PR machinery over score-sorted samples (ATen path + K3 dispatch).

Every curve metric reduces to per-row tie groups of the descending-sorted scores: at each
group end e we have cumulative TP_e, FP_e.  Then
  AUROC = sum_e (FP_e - FP_{e-1}) (TP_e + TP_{e-1}) / 2 / (P * N)   (0.5 if P * N == 0)
  AUPRC = sum_e (TP_e - TP_{e-1}) * TP_e / (TP_e + FP_e) / P        (0 if P == 0)
which equal the reference's trapz / Riemann sums over its compacted curves (auroc.py:115-152,
auprc.py + tensor_utils.py:12-16).  ROCm tensors use the fused K3 kernel; CPU tensors the
vectorised ATen form below (FP64 accumulation in both).
"""

from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F

from torcheval_amd.ops import use_native


def _group_ends(s: torch.Tensor) -> torch.Tensor:
    """Boolean mask of tie-group ends along the last dim of descending-sorted ``s``."""
    return F.pad(s[..., 1:] != s[..., :-1], (0, 1), value=True)


def _row_points(
    s: torch.Tensor, a: torch.Tensor, b: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """For one sorted row: thresholds, TP, FP at the tie-group ends (descending order)."""
    ends = _group_ends(s)
    tp = a.cumsum(-1)[ends]
    fp = b.cumsum(-1)[ends]
    return s[ends], tp, fp


def _areas_from_points(tp: torch.Tensor, fp: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    zero = tp.new_zeros(1)
    tp_prev = torch.cat([zero, tp[:-1]])
    fp_prev = torch.cat([zero, fp[:-1]])
    P = tp[-1] if tp.numel() else tp.new_zeros(())
    N = fp[-1] if fp.numel() else fp.new_zeros(())
    roc = ((fp - fp_prev) * (tp + tp_prev)).sum() / 2
    den = tp + fp
    prec = torch.where(den > 0, tp / torch.where(den > 0, den, torch.ones_like(den)), torch.zeros_like(den))
    pr = ((tp - tp_prev) * prec).sum()
    auroc = torch.where(P * N == 0, torch.full_like(roc, 0.5), roc / (P * N))
    auprc = torch.where(P == 0, torch.zeros_like(pr), pr / torch.where(P == 0, torch.ones_like(P), P))
    return auroc, auprc


def raw_area_sums(
    x: torch.Tensor, t: torch.Tensor, w: Optional[torch.Tensor], tp0: float, fp0: float
) -> torch.Tensor:
    """Un-normalised sums of one 1-D shard whose samples all rank below (TP0, FP0) worth of
    higher-scored samples held elsewhere: float64 [4] = (roc sum, pr sum, local P, local N)
    with roc = sum_i b_i (TPs + TPe) / 2 and pr = sum_i a_i TPe / (TPe + FPe) in GLOBAL counts.
    Summed over shards and divided by the global P * N (roc) or P (pr) they give AUROC / AUPRC.
    ROCm tensors run K3 with shard offsets; CPU tensors the ATen form."""
    if use_native(x) and t.is_cuda and x.numel() > 0:
        from torcheval_amd.ops.sortscan import binary_auc_raw

        return binary_auc_raw(x, t, w, tp0, fp0)
    dev = x.device
    if x.numel() == 0:
        return torch.zeros(4, dtype=torch.float64, device=dev)
    s, a, b = _sorted_ab(x.double() if x.dtype in (torch.float16, torch.bfloat16) else x, t, w)
    ends = _group_ends(s)
    tp = a.cumsum(-1)[ends] + tp0
    fp = b.cumsum(-1)[ends] + fp0
    tp_prev = torch.cat([tp.new_full((1,), tp0), tp[:-1]])
    fp_prev = torch.cat([fp.new_full((1,), fp0), fp[:-1]])
    roc = ((fp - fp_prev) * (tp + tp_prev)).sum() / 2
    den = tp + fp
    prec = torch.where(den > 0, tp / torch.where(den > 0, den, torch.ones_like(den)), torch.zeros_like(den))
    pr = ((tp - tp_prev) * prec).sum()
    return torch.stack([roc, pr, a.sum(), b.sum()]).to(torch.float64)


def _sorted_ab(
    x: torch.Tensor, t: torch.Tensor, w: Optional[torch.Tensor]
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    s, idx = torch.sort(x, dim=-1, descending=True)
    tt = t.gather(-1, idx).to(torch.float64)
    ww = torch.ones_like(tt) if w is None else w.gather(-1, idx).to(torch.float64)
    return s, ww * tt, ww * (1 - tt)


def binary_areas(
    input: torch.Tensor, target: torch.Tensor, weight: Optional[torch.Tensor] = None,
    *, roc: bool = True, pr: bool = False,
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """float64 [rows] AUROC / AUPRC of [rows, n] (or [n] -> [1]) binary data."""
    x = input if input.dim() == 2 else input.unsqueeze(0)
    t = target if target.dim() == 2 else target.unsqueeze(0)
    w = None if weight is None else (weight if weight.dim() == 2 else weight.unsqueeze(0))
    if use_native(x) and t.is_cuda and x.shape[-1] > 0:
        from torcheval_amd.ops.sortscan import binary_auc

        return binary_auc(x, t, w, roc=roc, pr=pr)
    rocs, prs = [], []
    s, a, b = _sorted_ab(x.to(torch.float64) if x.dtype in (torch.float16, torch.bfloat16) else x, t, w)
    for r in range(s.shape[0]):
        _, tp, fp = _row_points(s[r], a[r], b[r])
        ar, ap = _areas_from_points(tp, fp) if tp.numel() else (
            torch.tensor(0.5, dtype=torch.float64), torch.tensor(0.0, dtype=torch.float64))
        rocs.append(ar)
        prs.append(ap)
    dev = x.device
    return (torch.stack(rocs).to(dev) if roc else None, torch.stack(prs).to(dev) if pr else None)


def multiclass_areas(
    input: torch.Tensor, target: torch.Tensor, num_classes: int, *, roc: bool = True, pr: bool = False
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """float64 [C] one-vs-rest AUROC / AUPRC of [n, C] scores vs [n] labels."""
    if use_native(input) and target.is_cuda and input.shape[0] > 0:
        from torcheval_amd.ops.sortscan import multiclass_auc

        return multiclass_auc(input, target, roc=roc, pr=pr)
    onehot = (target[None, :] == torch.arange(num_classes, device=target.device)[:, None])
    return binary_areas(input.t(), onehot, None, roc=roc, pr=pr)


def pr_curve_row(
    s: torch.Tensor, a: torch.Tensor, b: torch.Tensor, out_dtype: torch.dtype = torch.float32
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Precision, recall, thresholds of one sorted row in the reference's layout: ascending
    thresholds, plus the final (precision=1, recall=0) point; recall is 1 when P == 0."""
    thr, tp, fp = _row_points(s, a, b)
    precision = (tp / (tp + fp)).flip(0).to(out_dtype)
    P = tp[-1]
    recall = (tp / P).flip(0).to(out_dtype)
    precision = torch.cat([precision, precision.new_ones(1)])
    recall = torch.cat([recall, recall.new_zeros(1)])
    if torch.isnan(recall[0]):
        recall = torch.nan_to_num(recall, 1.0)
    return precision, recall, thr.flip(0)


def pr_curves(
    x: torch.Tensor, t: torch.Tensor
) -> Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]:
    """Per-row PR curves of [rows, n] scores and {0,1} targets."""
    s, a, b = _sorted_ab(x, t, None)
    out_p, out_r, out_t = [], [], []
    for r in range(s.shape[0]):
        p, rc, th = pr_curve_row(s[r], a[r], b[r])
        out_p.append(p)
        out_r.append(rc)
        out_t.append(th)
    return out_p, out_r, out_t
