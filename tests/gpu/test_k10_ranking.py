"""K10 rank-of-target kernel (hit rate / reciprocal rank) vs the ATen path on CPU."""

import pytest
import torch

from torcheval_amd.metrics import HitRate, ReciprocalRank
from torcheval_amd.metrics.functional import hit_rate, reciprocal_rank
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,c", [(1, 1), (37, 5), (1000, 63), (4096, 64), (513, 130), (8192, 1000), (64, 5000)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_k10_matches_aten(n, c, dtype):
    assert native_loaded()
    g = torch.Generator().manual_seed(n * 7 + c)
    x = (torch.randint(0, 17, (n, c), generator=g).float() / 17).to(dtype)  # heavy ties
    if n > 3 and c > 3:
        x[1, 2] = float("nan")
        x[3].fill_(float("nan"))
    t = torch.randint(0, c, (n,), generator=g)
    for k in (None, 1, 3, c):
        if k is not None and k > 0:
            torch.testing.assert_close(hit_rate(x.cuda(), t.cuda(), k=k).cpu(), hit_rate(x, t, k=k))
        torch.testing.assert_close(reciprocal_rank(x.cuda(), t.cuda(), k=k).cpu(), reciprocal_rank(x, t, k=k))


def test_k10_strided_rows_and_int32_targets():
    g = torch.Generator().manual_seed(3)
    wide = torch.randn(500, 1031, generator=g)
    x = wide[:, 3:1003]  # unit column stride, row stride 1031, misaligned base
    t = torch.randint(0, 1000, (500,), generator=g, dtype=torch.int32)
    torch.testing.assert_close(reciprocal_rank(x.cuda(), t.cuda(), k=10).cpu(), reciprocal_rank(x, t.long(), k=10))
    torch.testing.assert_close(hit_rate(x.cuda(), t.cuda(), k=10).cpu(), hit_rate(x, t.long(), k=10))


def test_k10_class_metrics_and_bad_target():
    x = torch.randn(256, 100).cuda()
    t = torch.randint(0, 100, (256,)).cuda()
    m = ReciprocalRank(k=5).update(x, t).update(x, t)
    torch.testing.assert_close(m.compute().cpu(), torch.cat([reciprocal_rank(x.cpu(), t.cpu(), k=5)] * 2))
    h = HitRate(k=5).update(x, t)
    torch.testing.assert_close(h.compute().cpu(), hit_rate(x.cpu(), t.cpu(), k=5))
    bad = t.clone()
    bad[7] = 100
    m2 = ReciprocalRank().update(x, bad)
    with pytest.raises(RuntimeError, match="out of bounds"):
        m2.compute()
