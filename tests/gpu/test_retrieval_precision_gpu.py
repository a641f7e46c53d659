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
