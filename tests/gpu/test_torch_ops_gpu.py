"""torch.ops.torcheval_amd.* CUDA kernels through the dispatcher match the direct entry points."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_sort_and_rafp_through_dispatcher():
    from torcheval_amd.metrics.functional import binary_recall_at_fixed_precision

    x = torch.rand(1, 10_000, device=DEV)
    t = torch.randint(0, 2, (1, 10_000), device=DEV)
    s = torch.empty_like(x)
    o = torch.empty(1, 10_000, dtype=torch.int32, device=DEV)
    torch.ops.torcheval_amd.sort_desc(x, s, o, t.to(torch.uint8), 1)
    torch.testing.assert_close(s, torch.sort(x, dim=1, descending=True).values)
    rec = torch.empty(1, device=DEV)
    thr = torch.empty(1, device=DEV)
    torch.ops.torcheval_amd.rafp(s, o, t.to(torch.uint8), False, 1, 0.5, rec, thr)
    want = binary_recall_at_fixed_precision(x[0], t[0], min_precision=0.5)
    torch.testing.assert_close(rec[0], want[0])
    torch.testing.assert_close(thr[0], want[1])


def test_fid_cov_and_row_sums_through_dispatcher():
    a = torch.randn(300, 64, device=DEV)
    cov = torch.zeros(64, 64, device=DEV)
    col = torch.zeros(64, device=DEV)
    torch.ops.torcheval_amd.fid_cov_update(a, cov, col)
    torch.testing.assert_close(cov, a.T @ a, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(col, a.sum(0), rtol=1e-4, atol=1e-4)
    out = torch.zeros((), dtype=torch.float64, device=DEV)
    torch.ops.torcheval_amd.row_sums(a, None, None, 1.0, [out], [1], 1)
    torch.testing.assert_close(out, a.double().sum(), rtol=1e-9, atol=1e-6)
