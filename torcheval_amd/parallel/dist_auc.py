"""Sample-sharded exact AUROC / AUPRC across ranks (SURVEY.md §2.8 "SP analog", §5.7).

``sync_and_compute(BinaryAUROC)`` all-gathers every rank's samples and sorts the union on
every rank: O(N * world) memory per GPU.  For corpora too large for that (or to spread the
sort), ``distributed_binary_auroc`` keeps the samples sharded and uses the device-resident
collectives instead:

1. each rank contributes ``S`` evenly strided keys of its shard; one all-gather
   of the samples yields ``world - 1`` splitters (global quantiles);
2. every sample is routed to the rank owning its key range - ranks hold descending key ranges,
   rank 0 the highest - with ONE ``all_to_all_single`` per field over RCCL (the same exchange
   pattern as expert-parallel token routing).  Routing depends only on the key, so every tie
   group lands on one rank and no group straddles a shard boundary;
3. each rank sorts what it received (K3a), its (P_r, N_r) is all-gathered; rank r's scan starts at the (TP, FP) of all
   higher-key ranks (the K3 ``init`` offsets), so its per-sample ROC / PR terms are the global
   ones; one all-reduce of the 2 raw sums and a division by the global P * N (ROC) / P (PR)
   finishes.

Result: bit-for-bit the same tie-aware areas as the single-device computation (up to FP64
summation order), with per-rank memory O(N / world).
"""

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from torcheval_amd.metrics.functional.classification._curve import raw_area_sums
from torcheval_amd.parallel.collectives import _wait, skip_collectives
from torcheval_amd.parallel.distributed import transport_device

__all__ = ["distributed_binary_auroc", "distributed_binary_auprc", "distributed_binary_areas"]


def _order_key(x: torch.Tensor) -> torch.Tensor:
    # float -> a float64 whose order matches the K3a / torch.sort descending order: NaN first
    return torch.where(torch.isnan(x), torch.full_like(x, float("inf")), x).to(torch.float64)


def distributed_binary_areas(
    input: torch.Tensor,
    target: torch.Tensor,
    weight: Optional[torch.Tensor] = None,
    *,
    group: Optional[dist.ProcessGroup] = None,
    samples_per_rank: int = 256,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """(AUROC, AUPRC) as float64 scalars over the union of every rank's 1-D ``input``/``target``
    (and optional ``weight``) shards.  Collective: every rank of ``group`` must call it."""
    if input.dim() != 1 or target.shape != input.shape or (weight is not None and weight.shape != input.shape):
        raise ValueError("distributed_binary_areas expects 1-D input / target (/ weight) of equal shape")
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    dev = input.device
    if not dist.is_initialized() or skip_collectives(ws):
        raw = raw_area_sums(input, target, weight, 0.0, 0.0)
        return _normalise(raw[0], raw[1], raw[2], raw[3])
    tdev = transport_device(group)
    rank = dist.get_rank(group)

    # 1. splitters from S evenly strided samples of every rank's shard (a sample, not a sort:
    #    splitter quality only affects load balance, never the result); the trailing slot carries
    #    "this rank is weighted" so all ranks agree on the weight exchange for free
    keys = _order_key(input)
    n = keys.numel()
    S = samples_per_rank
    if n:
        samples = keys[torch.linspace(0, n - 1, S, device=dev).round().long()]
    else:
        samples = torch.full((S,), float("nan"), dtype=torch.float64, device=dev)
    flag = torch.full((1,), 1.0 if weight is not None else 0.0, dtype=torch.float64, device=dev)
    gathered = _all_gather_flat(torch.cat([samples, flag]).to(tdev), ws, group).view(ws, S + 1)
    any_weighted = bool(gathered[:, S].any())
    if any_weighted and weight is None:
        weight = torch.ones_like(input, dtype=torch.float64)
    pool = gathered[:, :S].reshape(-1)
    pool = pool[~torch.isnan(pool)].sort().values  # ascending
    if pool.numel() == 0:
        bounds = torch.zeros(ws - 1, dtype=torch.float64, device=tdev)
    else:
        q = (torch.arange(1, ws, device=tdev) * pool.numel()) // ws
        bounds = pool[q.clamp(max=pool.numel() - 1)]
    bounds = bounds.to(dev)

    # 2. route every sample to its key-range owner (rank 0 = highest keys)
    dest = (ws - 1) - torch.searchsorted(bounds, keys, right=True)
    order = torch.argsort(dest, stable=True)
    send_counts = torch.bincount(dest, minlength=ws)
    recv_counts = torch.empty_like(send_counts, device=tdev)
    _wait(dist.all_to_all_single(recv_counts, send_counts.to(tdev), group=group, async_op=True))
    send_splits = send_counts.tolist()
    recv_splits = recv_counts.cpu().tolist()
    total_recv = int(sum(recv_splits))

    def exchange(v: torch.Tensor) -> torch.Tensor:
        out = torch.empty(total_recv, dtype=v.dtype, device=tdev)
        _wait(dist.all_to_all_single(out, v[order].contiguous().to(tdev), recv_splits, send_splits,
                                     group=group, async_op=True))
        return out.to(dev)

    x_loc = exchange(input.to(torch.float32) if input.dtype in (torch.float16, torch.bfloat16) else input)
    t_loc = exchange(target.to(torch.float32))
    w_loc = exchange(weight.to(torch.float64)) if weight is not None else None

    # 3. shard totals -> offsets of all higher-key ranks, then the shard's raw sums
    wl = w_loc if w_loc is not None else torch.ones_like(t_loc, dtype=torch.float64)
    pn = torch.stack([(wl * t_loc.double()).sum(), (wl * (1 - t_loc.double())).sum()]).to(tdev)
    all_pn = _all_gather_flat(pn, ws, group).view(ws, 2).cpu()
    tp0, fp0 = (float(v) for v in all_pn[:rank].sum(0)) if rank > 0 else (0.0, 0.0)
    raw = raw_area_sums(x_loc, t_loc, w_loc, tp0, fp0).to(tdev)
    sums = raw[:2].clone()
    _wait(dist.all_reduce(sums, group=group, async_op=True))
    P, N = all_pn.sum(0).tolist()
    roc, pr = sums.to(dev).unbind(0)
    return _normalise(roc, pr, torch.tensor(P, dtype=torch.float64, device=dev),
                      torch.tensor(N, dtype=torch.float64, device=dev))


def _all_gather_flat(v: torch.Tensor, ws: int, group) -> torch.Tensor:
    out = torch.empty(ws * v.numel(), dtype=v.dtype, device=v.device)
    if v.is_cuda:
        _wait(dist.all_gather_into_tensor(out, v, group=group, async_op=True))  # one flat RCCL all-gather
    else:
        _wait(dist.all_gather(list(out.view(ws, -1).unbind(0)), v, group=group, async_op=True))
    return out


def _normalise(roc, pr, P, N) -> Tuple[torch.Tensor, torch.Tensor]:
    PN = P * N
    auroc = torch.where(PN == 0, torch.full_like(roc, 0.5), roc / torch.where(PN == 0, torch.ones_like(PN), PN))
    auprc = torch.where(P == 0, torch.zeros_like(pr), pr / torch.where(P == 0, torch.ones_like(P), P))
    return auroc, auprc


def distributed_binary_auroc(input, target, weight=None, *, group=None) -> torch.Tensor:
    """Exact tie-aware AUROC over every rank's shard without gathering the samples."""
    return distributed_binary_areas(input, target, weight, group=group)[0]


def distributed_binary_auprc(input, target, weight=None, *, group=None) -> torch.Tensor:
    """Exact AUPRC (average precision) over every rank's shard without gathering the samples."""
    return distributed_binary_areas(input, target, weight, group=group)[1]


def sharded_compute(metric, *, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """``compute()`` of a 1-task ``BinaryAUROC`` / ``BinaryAUPRC`` over every rank's samples with
    the sample-sharded algorithm above - the drop-in for ``sync_and_compute(metric)`` when the
    union of samples should not be materialised on every rank.  Returns on every rank."""
    from torcheval_amd.metrics.classification.auprc import BinaryAUPRC
    from torcheval_amd.metrics.classification.auroc import BinaryAUROC

    if not isinstance(metric, (BinaryAUROC, BinaryAUPRC)):
        raise TypeError(f"sharded_compute supports BinaryAUROC / BinaryAUPRC, got {type(metric).__name__}")
    if getattr(metric, "num_tasks", 1) != 1:
        raise ValueError("sharded_compute supports num_tasks == 1")
    dev = metric.device
    if metric.inputs:
        x = torch.cat([v.reshape(-1) for v in metric.inputs])
        t = torch.cat([v.reshape(-1) for v in metric.targets])
    else:
        x = torch.empty(0, device=dev)
        t = torch.empty(0, dtype=torch.long, device=dev)
    w = None
    if isinstance(metric, BinaryAUROC) and any(v.numel() for v in metric.weights):
        w = torch.cat([wv.reshape(-1) if wv.numel() else torch.ones_like(iv.reshape(-1), dtype=torch.float64)
                       for iv, wv in zip(metric.inputs, metric.weights)])
    roc, pr = distributed_binary_areas(x, t, w, group=group)
    return roc if isinstance(metric, BinaryAUROC) else pr.to(torch.float32)
