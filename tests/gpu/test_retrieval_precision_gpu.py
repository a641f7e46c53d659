"""Device-resident RetrievalPrecision on the GPU: identical results to the CPU path, and no
host synchronisation in update() / compute() (torch's sync debug mode turns any into an error)."""

import pytest
import torch

from torcheval_amd.metrics import RetrievalPrecision

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("k,limit,Q", [(None, False, 1000), (10, False, 1000), (10, True, 7), (1, False, 1)])
def test_retrieval_precision_gpu_matches_cpu_without_syncs(k, limit, Q):
    g = torch.Generator().manual_seed(Q + (k or 0))
    batches = []
    for n in (200_000, 1, 300_000):
        x = torch.rand(n, generator=g)
        t = torch.randint(0, 2, (n,), generator=g)
        idx = torch.randint(0, Q, (n,), generator=g)
        batches.append((x, t, idx))
    cpu = RetrievalPrecision(k=k, limit_k_to_size=limit, num_queries=Q, avg=None)
    gpu = RetrievalPrecision(k=k, limit_k_to_size=limit, num_queries=Q, avg=None, device=DEV)
    dev_batches = [(x.to(DEV), t.to(DEV), i.to(DEV)) for x, t, i in batches]
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for x, t, i in dev_batches:
            gpu.update(x, t, indexes=i if Q > 1 else None)
        out = gpu.compute()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    for x, t, i in batches:
        cpu.update(x, t, indexes=i if Q > 1 else None)
    torch.testing.assert_close(out.cpu(), cpu.compute(), equal_nan=True)
    assert out.is_cuda


def test_retrieval_precision_gpu_macro_and_empty_queries():
    m = RetrievalPrecision(k=2, num_queries=4, avg="macro", empty_target_action="skip", device=DEV)
    m.update(torch.tensor([0.9, 0.1, 0.8, 0.4], device=DEV), torch.tensor([1, 0, 0, 0], device=DEV),
             indexes=torch.tensor([0, 0, 1, 1], device=DEV))
    out = m.compute()
    # query 0: top-2 = (0.9: 1, 0.1: 0) -> 0.5; query 1: no positive -> skip; 2, 3: empty
    torch.testing.assert_close(out.cpu(), torch.tensor(0.5))


@pytest.mark.parametrize("k,Q", [(1, 1), (5, 3), (10, 1000), (64, 37), (3, 5000)])
def test_k10b_state_matches_sort_path(k, Q, monkeypatch):
    """K10b (retrieval.hip) and the sort-based ATen path leave identical state rows on
    tie-free scores, out-of-range query ids included."""
    import torcheval_amd.ops as ops

    g = torch.Generator().manual_seed(k * 7919 + Q)
    batches = []
    for n in (50_000, 0, 3, 120_000):
        x = torch.randperm(1 << 22, generator=g)[:n].float() / (1 << 22)  # distinct scores
        t = torch.randint(0, 3, (n,), generator=g)
        idx = torch.randint(-1, Q + 1, (n,), generator=g)
        batches.append((x.to(DEV), t.to(DEV), idx.to(DEV)))
    nat = RetrievalPrecision(k=k, num_queries=Q, device=DEV)
    ref = RetrievalPrecision(k=k, num_queries=Q, device=DEV)
    for x, t, i in batches:
        nat.update(x, t, indexes=i if Q > 1 else None)
        monkeypatch.setattr(ops, "DISABLE_HIP", True)
        ref.update(x, t, indexes=i if Q > 1 else None)
        monkeypatch.setattr(ops, "DISABLE_HIP", False)
        torch.testing.assert_close(nat.topk, ref.topk, rtol=0, atol=0)
        torch.testing.assert_close(nat.target, ref.target.to(nat.target.dtype), rtol=0, atol=0)
        assert torch.equal(nat.count, ref.count)
    torch.testing.assert_close(nat.compute(), ref.compute(), equal_nan=True)


@pytest.mark.parametrize("k,Q", [(1, 1), (5, 3), (64, 37)])
def test_k10b_ties_keep_cat_order(k, Q):
    """Ties (quantised scores, NaN, -0 vs +0, -inf) resolve in the reference's cat order: old
    row entries first, then batch order - a stable descending sort of cat(old, batch) per
    query (NaN highest), computed here on the host as the oracle."""
    g = torch.Generator().manual_seed(k + 31 * Q)
    m = RetrievalPrecision(k=k, num_queries=Q, device=DEV)
    rows_v = [torch.empty(0) for _ in range(Q)]
    rows_t = [torch.empty(0) for _ in range(Q)]
    for n in (4000, 17, 6000):
        x = (torch.randint(0, 8, (n,), generator=g) / 8.0).float()
        x[:4] = torch.tensor([float("nan"), -0.0, 0.0, float("-inf")])
        t = torch.randint(0, 5, (n,), generator=g).float()
        idx = torch.randint(-1, Q + 1, (n,), generator=g)
        m.update(x.to(DEV), t.to(DEV), indexes=idx.to(DEV) if Q > 1 else None)
        for q in range(Q):
            sel = (idx == q) if Q > 1 else torch.ones(n, dtype=torch.bool)
            v = torch.cat([rows_v[q], x[sel]])
            tt = torch.cat([rows_t[q], t[sel]])
            key = torch.where(torch.isnan(v), torch.full_like(v, float("inf")), v)
            nan_first = torch.isnan(v).float()
            # stable descending by (is-nan, value): sort by value first, then by nan flag
            o1 = torch.sort(key, descending=True, stable=True).indices
            o = o1[torch.sort(nan_first[o1], descending=True, stable=True).indices]
            rows_v[q], rows_t[q] = v[o][:k], tt[o][:k]
    for q in range(Q):
        c = rows_v[q].numel()
        torch.testing.assert_close(m.topk[q, :c].cpu(), rows_v[q], equal_nan=True, rtol=0, atol=0)
        torch.testing.assert_close(m.target[q, :c].cpu(), rows_t[q], rtol=0, atol=0)
        assert int(m.count[q]) == c
