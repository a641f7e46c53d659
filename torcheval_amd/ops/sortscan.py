"""K3 sort-and-scan wrappers (csrc/kernels/sortscan.hip): exact tie-aware AUROC / AUPRC.

Pipeline per call: one segmented device sort of the scores (descending, one row per task /
class) followed by the four-launch K3 scan.  No host synchronisation anywhere.
"""

from typing import Optional, Tuple

import torch

from torcheval_amd.ops import native


def _sort_rows(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    if x.dtype not in (torch.float32, torch.float64):
        x = x.float()  # f16/bf16 -> f32 is exact and order preserving
    s, idx = torch.sort(x.contiguous(), dim=-1, descending=True)
    return s, idx


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
    s, idx = _sort_rows(x)
    rows = s.shape[0]
    out_roc = torch.empty(rows, dtype=torch.float64, device=x.device) if roc else None
    out_pr = torch.empty(rows, dtype=torch.float64, device=x.device) if pr else None
    native().auc_scan(s, idx, t, w, False, out_roc, out_pr)
    return out_roc, out_pr


def multiclass_auc(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    roc: bool = True,
    pr: bool = False,
) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """One-vs-rest per-class AUROC / AUPRC (float64 [C]) of ``input`` [n, C] vs labels [n]."""
    s, idx = _sort_rows(input.t())
    rows = s.shape[0]
    out_roc = torch.empty(rows, dtype=torch.float64, device=input.device) if roc else None
    out_pr = torch.empty(rows, dtype=torch.float64, device=input.device) if pr else None
    native().auc_scan(s, idx, target, None, True, out_roc, out_pr)
    return out_roc, out_pr
