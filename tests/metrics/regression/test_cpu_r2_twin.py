"""The small-batch CPU host twin of the functional r2_score (cpu_metrics.cpp cpu_r2) against the
ATen form: 1-D / 2-D, float32 / float64, all three multioutput modes, adjusted R2; dtype and
shape exact, values to FP rounding; the reference's sample-count errors still raised."""
import importlib

import pytest
import torch

from torcheval_amd.metrics.functional import r2_score
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="extension not built")
MOD = importlib.import_module("torcheval_amd.metrics.functional.regression.r2_score")


@pytest.mark.parametrize("shape", [(8,), (8, 4), (2,), (100, 3)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("mo", ["uniform_average", "raw_values", "variance_weighted"])
@pytest.mark.parametrize("k", [0, 1])
def test_twin_matches_aten(monkeypatch, shape, dtype, mo, k):
    if k >= shape[0] - 1:
        pytest.skip("needs more samples than regressors + 1")
    g = torch.Generator().manual_seed(shape[0] * 3 + len(shape))
    x = torch.randn(*shape, generator=g).to(dtype)
    t = (torch.randn(*shape, generator=g) + 1).to(dtype)
    assert MOD._cpu_r2_ok(x, t)
    got = r2_score(x, t, multioutput=mo, num_regressors=k)
    monkeypatch.setattr(MOD, "_cpu_r2_ok", lambda *a: False)
    want = r2_score(x, t, multioutput=mo, num_regressors=k)
    assert got.dtype == want.dtype and got.shape == want.shape
    torch.testing.assert_close(got, want, rtol=2e-5, atol=1e-6)


def test_errors_still_raised():
    with pytest.raises(ValueError, match="at least two samples"):
        r2_score(torch.rand(1), torch.rand(1))
    with pytest.raises(ValueError, match="num_regressors"):
        r2_score(torch.rand(4), torch.rand(4), num_regressors=3)
