"""Cancellation-prone R2 / MSE inputs (near-constant and large-offset targets).

The native paths (the CPU twins for <= 65536 elements, K5 on ROCm) accumulate the sums in FP64
and round each sum ONCE to float32, then apply the reference's float32 formula
(tss = sso - so^2 / n, r2 = 1 - rss / tss).  The ATen path - and the reference - accumulate the
sums in float32, so their sums depend on the summation order.  With cancellation in tss a
one-ULP difference in a sum can move r2 far (docs/parity.md), so the two paths can disagree on
such data; what the native path guarantees is pinned here: its result is exactly the
reference formula applied to the correctly rounded sums, whatever the batch order."""

import pytest
import torch

from torcheval_amd.metrics.functional import mean_squared_error, r2_score
from torcheval_amd.metrics.functional.regression.r2_score import _r2_score_compute, _r2_score_update
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="native build absent")


def _formula_on_rounded_sums(x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    xd, td = x.double(), t.double()
    sso = (td * td).sum(0).float()
    so = td.sum(0).float()
    rss = ((td - xd) ** 2).sum(0).float()
    return _r2_score_compute(sso, so, rss, torch.tensor(t.shape[0]), "raw_values", 0)


@pytest.mark.parametrize("offset,spread", [(1e3, 1e-2), (1e4, 1.0), (-3e3, 5e-2), (0.0, 1.0)])
@pytest.mark.parametrize("shape", [(4096,), (2048, 3)])
def test_r2_twin_is_the_formula_on_correctly_rounded_sums(offset, spread, shape):
    g = torch.Generator().manual_seed(int(abs(offset)) + shape[0])
    t = (offset + spread * torch.randn(shape, generator=g)).float()
    x = (t + 0.3 * spread * torch.randn(shape, generator=g)).float()
    twin = r2_score(x, t, multioutput="raw_values")
    torch.testing.assert_close(twin, _formula_on_rounded_sums(x, t), rtol=0, atol=0, equal_nan=True)
    # the batch order does not change the native result (the float32 ATen sums may)
    perm = torch.randperm(shape[0], generator=g)
    torch.testing.assert_close(r2_score(x[perm], t[perm], multioutput="raw_values"), twin, rtol=0, atol=0,
                               equal_nan=True)
    if offset == 0.0:  # well conditioned: every path agrees
        aten = _r2_score_compute(*_r2_score_update(x, t), "raw_values", 0)
        torch.testing.assert_close(twin, aten, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("offset", [1e3, 1e5])
def test_mse_twin_matches_the_exact_value(offset):
    g = torch.Generator().manual_seed(7)
    t = (offset + torch.randn(8192, generator=g)).float()
    x = (t + 0.01 * torch.randn(8192, generator=g)).float()
    exact = float(((t.double() - x.double()) ** 2).mean())
    assert abs(float(mean_squared_error(x, t)) - exact) <= 1e-6 * exact
