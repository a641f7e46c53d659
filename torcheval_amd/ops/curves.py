"""K3c wrappers (csrc/kernels/curves.hip): precision-recall curves and recall at fixed
precision on ROCm, batched over rows (classes / labels).

PR curves: K3a sort (payload-carrying) -> count + scan -> ONE host read of the per-row group
counts (the reference's single ``.tolist()``) -> emission straight into the exact, contiguous
outputs, split into per-row views.  Recall at fixed precision: the same passes plus a device
search, with no host synchronisation at all.
"""

from typing import List, Optional, Tuple

import torch

from torcheval_amd.ops import native
from torcheval_amd.ops.hostread import read_ints
from torcheval_amd.ops.sortscan import PAYLOAD_LABEL, PAYLOAD_TARGET, _sort_rows

Curves = Tuple[List[torch.Tensor], List[torch.Tensor], List[torch.Tensor]]


def _rows_major(x: torch.Tensor) -> torch.Tensor:
    """[n, c] scores -> [c, n] rows (LDS-tiled transpose for f32)."""
    if x.dtype in (torch.float16, torch.bfloat16):
        x = x.float()
    if x.dtype == torch.float32 and x.stride(-1) == 1 and x.shape[0] > 0:
        xt = torch.empty(x.shape[1], x.shape[0], dtype=torch.float32, device=x.device)
        native().transpose_f32(x, xt)
        return xt
    return x.t()


def _prepare(x: torch.Tensor, payload: torch.Tensor, kind: int):
    """Sort the rows descending; f32 keys carry the payload through K3a, f64 keys go through
    torch.sort (kind 0: K3c gathers the targets through the permutation)."""
    if x.dtype not in (torch.float32, torch.float64):
        x = x.float()
    return _sort_rows(x, payload, kind)


def _curves(x: torch.Tensor, payload: torch.Tensor, kind: int, class_mode: bool, out_dtype: torch.dtype) -> Curves:
    s, idx, k = _prepare(x, payload, kind)
    rows, n = s.shape
    dev = s.device
    target = payload  # read by K3c only for f64 keys (kind 0): gathered through the permutation
    ws = torch.empty(native().curve_workspace_bytes(rows, n, False), dtype=torch.uint8, device=dev)
    sizes = torch.empty(rows, dtype=torch.int64, device=dev)
    native().curve_count(s, idx, target, class_mode, k, ws, sizes)
    row_off = sizes.cumsum(0) - sizes
    sz = read_ints(sizes)  # the one host synchronisation (pinned-memory path for <= 7 rows)
    total = int(sum(sz))
    prec = torch.empty(total + rows, dtype=torch.float32, device=dev)
    rec = torch.empty(total + rows, dtype=torch.float32, device=dev)
    thr = torch.empty(total, dtype=s.dtype, device=dev)
    native().curve_emit(s, idx, target, class_mode, k, ws, sizes, row_off, prec, rec, thr)
    if thr.dtype != out_dtype:
        thr = thr.to(out_dtype)
    pts = [g + 1 for g in sz]
    return list(prec.split(pts)), list(rec.split(pts)), list(thr.split(sz))


def binary_pr_curve(input: torch.Tensor, target: torch.Tensor, pos_label: int = 1) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Ascending-threshold PR curve of [n] scores (positives: target == pos_label)."""
    pos = (target == pos_label).to(torch.uint8).reshape(1, -1)
    p, r, t = _curves(input.reshape(1, -1), pos, PAYLOAD_TARGET, False, input.dtype)
    return p[0], r[0], t[0]


def multiclass_pr_curves(input: torch.Tensor, target: torch.Tensor) -> Curves:
    """One-vs-rest PR curves of [n, C] scores vs [n] labels (one batched pass over C rows)."""
    labels = target if target.dtype in (torch.int32, torch.int64) else target.long()
    return _curves(_rows_major(input), labels, PAYLOAD_LABEL, True, input.dtype)


def multilabel_pr_curves(input: torch.Tensor, target: torch.Tensor) -> Curves:
    """Per-label PR curves of [n, L] scores vs [n, L] {0, 1} targets (positives: target == 1)."""
    pos = (target == 1).t()  # [L, n] view; _sort_rows lays it out once (fast transpose)
    return _curves(_rows_major(input), pos, PAYLOAD_TARGET, False, input.dtype)


def _rafp(x: torch.Tensor, payload: torch.Tensor, kind: int, class_mode: bool, min_precision: float,
          out_dtype: torch.dtype) -> Tuple[torch.Tensor, torch.Tensor]:
    s, idx, k = _prepare(x, payload, kind)
    rows = s.shape[0]
    target = payload
    rec = torch.empty(rows, dtype=torch.float32, device=s.device)
    thr = torch.empty(rows, dtype=s.dtype, device=s.device)
    native().rafp(s, idx, target, class_mode, k, float(min_precision), rec, thr)
    return rec, thr.to(out_dtype) if thr.dtype != out_dtype else thr


def binary_rafp(input: torch.Tensor, target: torch.Tensor, min_precision: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """(max recall with precision >= min_precision, its |threshold|) as 0-d tensors, sync-free."""
    pos = (target == 1).to(torch.uint8).reshape(1, -1)
    rec, thr = _rafp(input.reshape(1, -1), pos, PAYLOAD_TARGET, False, min_precision,
                     torch.promote_types(input.dtype, torch.float32))
    return rec[0], thr[0]


def multilabel_rafp(input: torch.Tensor, target: torch.Tensor, min_precision: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-label (max recall [L], |best threshold| [L]) of [n, L] data, sync-free."""
    pos = (target == 1).t()  # [L, n] view; _sort_rows lays it out once (fast transpose)
    return _rafp(_rows_major(input), pos, PAYLOAD_TARGET, False, min_precision,
                 torch.promote_types(input.dtype, torch.float32))
