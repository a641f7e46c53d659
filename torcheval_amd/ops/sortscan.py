"""K3 sort-and-scan wrappers (csrc/kernels/sortscan.hip): exact tie-aware AUROC / AUPRC.

Pipeline per call: one segmented device sort of the scores (descending, one row per task /
class) followed by the K3 scan.  Opt-in (``TORCHEVAL_AMD_K3_FOLD=1``): with a target / label
payload on the onesweep sort, the sort's last pass also folds the scan's 1024-sample tile totals,
so the scan skips its tile_sums launch (7 launches for binary_auroc at 1M; measured slower, see
``_FOLD``).  No host synchronisation anywhere.  (A bucketed
no-global-sort variant, K3b, was built and measured slower at every size - see
profiles/README.md, round 3 - and removed.)
"""

import os
from typing import Optional, Tuple

import torch

from torcheval_amd.ops import native


PAYLOAD_TARGET, PAYLOAD_LABEL = 1, 2
_TARGET_PAYLOAD = (torch.float32, torch.int64, torch.int32, torch.uint8, torch.bool)


def _rows_f32(v: torch.Tensor) -> torch.Tensor:
    """A [rows, n] operand with unit stride along samples, as float32 values.  The transposed
    view of a row-major [n, rows] tensor (multilabel scores / targets) goes through the LDS-tiled
    ``transpose_f32`` (ATen's strided copy of such a view is ~10x slower)."""
    if v.dim() == 2 and v.stride(-1) != 1 and v.stride(0) == 1 and v.t().is_contiguous() and v.numel() > 0:
        src = v.t() if v.dtype == torch.float32 else v.t().float()
        out = torch.empty(v.shape, dtype=torch.float32, device=v.device)
        native().transpose_f32(src, out)
        return out
    return v if v.dtype == torch.float32 and v.stride(-1) == 1 else v.float().contiguous()


# TORCHEVAL_AMD_K3_FOLD=1: the onesweep sort's last pass folds the scan's tile totals (7 launches
# for binary_auroc at 1M instead of 8).  Off by default: measured slower - 88.8 vs 82.6 us at 1M,
# the fold's device atomics cost ~8 us against the ~4 us of the tile_sums launch they remove
# (profiles/k3_fold_r5.json)
_FOLD = os.environ.get("TORCHEVAL_AMD_K3_FOLD", "0") == "1"


def _fold_buffer(x: torch.Tensor) -> Optional[torch.Tensor]:
    """float64 [rows, ceil(n / 1024), 2] for the sort's tile-sum fold (uninitialised: the sort
    zeroes it in its first pass)."""
    rows, n = (1, x.shape[0]) if x.dim() == 1 else (x.shape[0], x.shape[-1])
    return torch.empty(rows, (n + 1023) // 1024, 2, dtype=torch.float64, device=x.device)


def _sort_rows(
    x: torch.Tensor, payload: Optional[torch.Tensor] = None, payload_kind: int = 0
) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """Descending per-row sort -> (sorted, order, kind); see ``_sort_rows_fold``."""
    return _sort_rows_fold(x, payload, payload_kind, False)[:3]


def _sort_rows_fold(
    x: torch.Tensor, payload: Optional[torch.Tensor] = None, payload_kind: int = 0, fold: bool = True
) -> Tuple[torch.Tensor, torch.Tensor, int, Optional[torch.Tensor]]:
    """Descending per-row sort -> (sorted, order, kind, tile sums or None).

    f32 runs the K3a radix sort.  With ``payload`` it carries the per-sample target
    (``PAYLOAD_TARGET``: f32 value) or class label (``PAYLOAD_LABEL``: int32; a 1-D payload is
    shared by every row) through the sort instead of the source index, so K3 reads targets in
    sorted order without a random gather (``kind`` echoes what ``order`` holds); then the sort
    may also return the scan's tile totals (``auc_scan(tsum=...)``).  f64 keys go through
    torch.sort (int64 permutation, kind 0)."""
    if x.dtype not in (torch.float32, torch.float64):
        x = x.float()  # f16/bf16 -> f32 is exact and order preserving
    if x.dtype == torch.float32 and x.shape[-1] < 2**31:
        if x.stride(-1) != 1:
            x = _rows_f32(x)
        s = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        idx = torch.empty(x.shape, dtype=torch.int32, device=x.device)
        kind = payload_kind if payload is not None else 0
        if kind == PAYLOAD_TARGET and (payload.dtype not in _TARGET_PAYLOAD or
                                       (payload.dim() == 2 and payload.stride(-1) != 1)):
            # K3a converts a target payload to its f32 value anyway
            payload = _rows_f32(payload)
        elif kind == PAYLOAD_LABEL and payload.dtype not in (torch.int64, torch.int32):
            payload = payload.long()
        buf = _fold_buffer(x) if fold and _FOLD and kind != 0 else None
        folded = native().sort_desc(x, s, idx, payload, kind, buf)
        return s, idx, kind, buf if folded else None
    s, idx = torch.sort(x.contiguous(), dim=-1, descending=True)
    return s, idx, 0, None


def binary_auc(
    input: torch.Tensor,
    target: torch.Tensor,
    weight: Optional[torch.Tensor] = None,
    *,
    roc: bool = True,
    pr: bool = False,
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Per-row AUROC / AUPRC (float64 [rows]) of ``input``/``target`` shaped [rows, n]."""
    x = input if input.dim() == 2 else input.unsqueeze(0)
    t = target if target.dim() == 2 else target.unsqueeze(0)
    w = None
    if weight is not None:
        w = weight if weight.dim() == 2 else weight.unsqueeze(0)
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    s, idx, kind, tsum = _sort_rows_fold(x, t if w is None else None, PAYLOAD_TARGET)
    rows = s.shape[0]
    out_roc = torch.empty(rows, dtype=torch.float64, device=x.device) if roc else None
    out_pr = torch.empty(rows, dtype=torch.float64, device=x.device) if pr else None
    native().auc_scan(s, idx, t, w, False, out_roc, out_pr, None, None, kind, tsum)
    return out_roc, out_pr


def multiclass_auc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    roc: bool = True,
    pr: bool = False,
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """One-vs-rest per-class AUROC / AUPRC (float64 [C]) of ``input`` [n, C] vs labels [n]."""
    x = input
    if x.dtype in (torch.float16, torch.bfloat16):
        x = x.float()
    if x.dtype == torch.float32 and x.stride(-1) == 1:
        xt = torch.empty(x.shape[1], x.shape[0], dtype=torch.float32, device=x.device)
        native().transpose_f32(x, xt)  # LDS-tiled; torch's strided copy is ~10x slower here
    else:
        xt = x.t()
    s, idx, kind, tsum = _sort_rows_fold(xt, target, PAYLOAD_LABEL)
    rows = s.shape[0]
    out_roc = torch.empty(rows, dtype=torch.float64, device=input.device) if roc else None
    out_pr = torch.empty(rows, dtype=torch.float64, device=input.device) if pr else None
    native().auc_scan(s, idx, target, None, True, out_roc, out_pr, None, None, kind, tsum)
    return out_roc, out_pr


def binary_auc_raw(
    input: torch.Tensor, target: torch.Tensor, weight: Optional[torch.Tensor], tp0: float, fp0: float
) -> torch.Tensor:
    """K3 over one 1-D shard with global (TP, FP) offsets: float64 [4] = (roc sum, pr sum,
    local P, local N) - see ``_curve.raw_area_sums``."""
    x = input.reshape(1, -1)
    t = target.reshape(1, -1)
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    w = None if weight is None else weight.reshape(1, -1)
    s, idx, kind, tsum = _sort_rows_fold(x, t if w is None else None, PAYLOAD_TARGET)
    init = torch.tensor([[tp0, fp0]], dtype=torch.float64, device=x.device)
    raw = torch.empty(1, 4, dtype=torch.float64, device=x.device)
    native().auc_scan(s, idx, t, w, False, None, None, init, raw, kind, tsum)
    return raw[0]
