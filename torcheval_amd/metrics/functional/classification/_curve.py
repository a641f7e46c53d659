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

from torcheval_amd.ops import compiling, native_loaded, use_native


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
    if _cpu_auc_ok(x, t, w):
        # small CPU batches: one C++ pass per row (sort + tie-group scan) instead of ~15 ATen
        # dispatches per row
        from torcheval_amd.ops import native

        r_, p_ = native().cpu_binary_auc(x, t, w)
        return (r_ if roc else None, p_ if pr else None)
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


_CPU_AUC_MAX = 1 << 16
_CPU_AUC_TARGETS = (torch.bool, torch.uint8, torch.int32, torch.int64, torch.float32, torch.float64)


def _cpu_auc_ok(x: torch.Tensor, t: torch.Tensor, w: Optional[torch.Tensor]) -> bool:
    return (
        not x.is_cuda
        and x.device.type == "cpu"
        and x.numel() <= _CPU_AUC_MAX
        and x.dtype in (torch.float32, torch.float64)
        and t.dtype in _CPU_AUC_TARGETS
        and (w is None or w.dtype in (torch.float32, torch.float64))
        and not compiling()
        and native_loaded()
    )


def multiclass_areas(
    input: torch.Tensor, target: torch.Tensor, num_classes: int, *, roc: bool = True, pr: bool = False
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """float64 [C] one-vs-rest AUROC / AUPRC of [n, C] scores vs [n] labels."""
    if use_native(input) and target.is_cuda and input.shape[0] > 0:
        from torcheval_amd.ops.sortscan import multiclass_auc

        return multiclass_auc(input, target, roc=roc, pr=pr)
    onehot = (target[None, :] == torch.arange(num_classes, device=target.device)[:, None])
    return binary_areas(input.t(), onehot, None, roc=roc, pr=pr)


def _tie_tails(s: torch.Tensor) -> torch.Tensor:
    """Tie-group tails of descending-sorted rows with the reference's ``diff != 0`` test (so
    adjacent infinities and NaNs end their own groups, exactly as in precision_recall_curve.py)."""
    return F.pad(s.diff(dim=-1) != 0, (0, 1), value=True)


def _curve_tables(x: torch.Tensor, pos: torch.Tensor):
    """Per-row descending sort -> (sorted keys, tails mask, precision, recall) over every
    sample of [rows, n]; precision / recall are the reference's int64 / int64 float32 values
    (recall 1 for a row without positives, the reference's nan_to_num)."""
    s, idx = torch.sort(x, dim=-1, descending=True)
    hit = pos.gather(-1, idx)
    tp = hit.cumsum(-1)
    fp = (~hit).cumsum(-1)
    precision = tp / (tp + fp)
    recall = (tp / tp[..., -1:]).nan_to_num_(1.0)
    return s, _tie_tails(s), precision, recall


def pr_curves(x: torch.Tensor, pos: torch.Tensor) -> Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]:
    """Per-row PR curves of [rows, n] scores and boolean positives, reference layout: ascending
    thresholds, then the final (precision 1, recall 0) point.  All rows in one vectorised pass,
    one host read of the per-row sizes (ATen path; ROCm tensors take K3c, ops/curves.py)."""
    s, tails, precision, recall = _curve_tables(x, pos)
    tails = tails.flip(-1)
    rows = s.shape[0]
    sizes = tails.sum(-1).tolist()
    thr = s.flip(-1)[tails].split(sizes)
    keep = F.pad(tails, (0, 1), value=True)
    one = precision.new_ones(rows, 1)
    prec = torch.cat([precision.flip(-1), one], -1)[keep].split([g + 1 for g in sizes])
    rec = torch.cat([recall.flip(-1), one.zero_()], -1)[keep].split([g + 1 for g in sizes])
    return list(prec), list(rec), list(thr)


def recall_at_precision_rows(
    x: torch.Tensor, pos: torch.Tensor, min_precision: float
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per row of [rows, n]: (max recall over curve points with precision >= min_precision,
    |highest threshold among the points reaching it|), the appended (1, 0) point included with
    threshold -1 (recall_at_fixed_precision.py:131-141 semantics), vectorised over rows with no
    host synchronisation."""
    s, tails, precision, recall = _curve_tables(x, pos)
    if not s.is_floating_point():  # the reference's cat with the float -1 promotes
        s = s.float()
    rows = s.shape[0]
    p = torch.tensor(min_precision, dtype=precision.dtype)
    qual = tails & (precision >= p)
    zero = recall.new_zeros(rows, 1)
    max_recall = torch.cat([torch.where(qual, recall, recall.new_full((), -1.0)), zero], -1).amax(-1)
    hit = tails & (recall == max_recall[:, None])
    neg_inf = torch.tensor(float("-inf"), dtype=s.dtype)
    cand = torch.where(hit, s, neg_inf)
    best = cand.amax(-1)  # a NaN candidate propagates, as in the reference's torch.max
    best = torch.where(max_recall == 0, torch.maximum(best, torch.full_like(best, -1.0)), best)
    return max_recall, best.abs()


# ---------------------------------------------------------------- sorted runs
def sort_run(x: torch.Tensor, t: torch.Tensor, w: Optional[torch.Tensor]):
    """One 1-D sample set sorted descending (NaN first, as K3a / torch.sort): (scores, targets,
    weights) permuted together - the form a rank ships to a distributed sync, so the receiver
    merges sorted runs instead of sorting the union.  Unweighted ROCm runs with bool / integer /
    f32 targets carry the target through the K3a sort as its f32 value (no permutation gather;
    the shipped targets are then f32 - exact for every 0/1 label), which is also the payload
    the receiver's merge carries."""
    if use_native(x) and x.dtype == torch.float32 and x.numel() > 0:
        from torcheval_amd.ops.sortscan import PAYLOAD_TARGET, _sort_rows

        if w is None and x.is_cuda and t.dtype in (torch.bool, torch.uint8, torch.int32, torch.int64, torch.float32):
            tp = t.to(torch.uint8) if t.dtype == torch.bool else t
            s, idx, kind = _sort_rows(x.reshape(1, -1), tp.reshape(1, -1), PAYLOAD_TARGET)
            if kind == PAYLOAD_TARGET:
                return s[0], idx[0].view(torch.float32), None
            return s[0], t[idx[0].long()], None
        s, idx, _ = _sort_rows(x.reshape(1, -1))
        perm = idx[0].long()
        s = s[0]
    else:
        s, perm = torch.sort(x, descending=True, stable=True)
    return s, t[perm], (None if w is None else w[perm])


def merged_areas(runs_x, runs_t, runs_w, *, roc: bool, pr: bool):
    """float64 (AUROC, AUPRC) of the union of 1-D runs that are each sorted descending: the
    runs are merged (K3m merge path on ROCm, a host merge on CPU; log2(R) passes, the first
    reading the runs in place) and the merged order feeds the K3 scan directly - no sort of
    the union.  Unweighted ROCm runs carry their targets (as f32) through the merge, so K3
    reads them in order without a gather (the K3a ``PAYLOAD_TARGET`` convention)."""
    from torcheval_amd.ops import native
    from torcheval_amd.ops.sortscan import PAYLOAD_TARGET

    xs = [r.reshape(-1).contiguous() for r in runs_x]
    if xs[0].is_cuda and use_native(xs[0]) and runs_w is None:
        pays = [r.reshape(-1).to(torch.float32).contiguous() for r in runs_t]
        if len(xs) == 1:  # one run is already merged
            s, p = xs[0], pays[0].view(torch.int32)
        else:
            s, p = native().merge_sorted_runs(xs, pays)
        out_roc = torch.empty(1, dtype=torch.float64, device=s.device) if roc else None
        out_pr = torch.empty(1, dtype=torch.float64, device=s.device) if pr else None
        native().auc_scan(s[None], p[None], p.view(torch.float32)[None], None, False, out_roc, out_pr, None, None,
                          PAYLOAD_TARGET)
        return out_roc, out_pr
    t = torch.cat([r.reshape(-1) for r in runs_t])
    w = None if runs_w is None else torch.cat([r.reshape(-1) for r in runs_w])
    gpu = xs[0].is_cuda and use_native(xs[0])  # False under DISABLE_HIP: no GPU kernel then
    if gpu or (not xs[0].is_cuda and native_loaded()):
        s, order = native().merge_sorted_runs(xs)  # K3m on ROCm, the C++ host merge on CPU
    else:  # ATen: a stable sort of the concatenation is the rank-ordered merge
        s, order = torch.sort(torch.cat(xs), descending=True, stable=True)
    if gpu and t.is_cuda:
        tt = t if t.dtype != torch.bool else t.to(torch.uint8)
        out_roc = torch.empty(1, dtype=torch.float64, device=s.device) if roc else None
        out_pr = torch.empty(1, dtype=torch.float64, device=s.device) if pr else None
        native().auc_scan(s[None], order[None], tt[None], None if w is None else w[None], False,
                          out_roc, out_pr, None, None, 0)
        return out_roc, out_pr
    o = order.long()
    tt = t[o].to(torch.float64)
    ww = torch.ones_like(tt) if w is None else w[o].to(torch.float64)
    _, tp, fp = _row_points(s, ww * tt, ww * (1 - tt))
    ar, ap = _areas_from_points(tp, fp) if tp.numel() else (
        torch.tensor(0.5, dtype=torch.float64), torch.tensor(0.0, dtype=torch.float64))
    return (ar.reshape(1) if roc else None, ap.reshape(1) if pr else None)


def runs_mergeable(metric, inputs) -> bool:
    """Whether a sample-store metric's list states are sorted runs the merge path can take."""
    return (
        getattr(metric, "_sorted_runs", False)
        and len(inputs) >= 1
        and all(x.dim() == 1 and x.dtype == torch.float32 for x in inputs)
    )
