"""The small-batch CPU host twin of the functional mean_squared_error (cpu_metrics.cpp cpu_mse)
against the ATen form: 1-D / 2-D, float32 / float64, unweighted, weighted, weights summing to
(almost) zero, both multioutput modes; output dtype and shape exact, values to FP rounding."""
import importlib

import pytest
import torch

from torcheval_amd.metrics.functional import mean_squared_error
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="extension not built")
MOD = importlib.import_module("torcheval_amd.metrics.functional.regression.mean_squared_error")


@pytest.mark.parametrize("shape", [(8,), (8, 4), (1,), (100, 3)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("weight", ["none", "rand", "tiny_negative"])
@pytest.mark.parametrize("mo", ["uniform_average", "raw_values"])
def test_twin_matches_aten(monkeypatch, shape, dtype, weight, mo):
    g = torch.Generator().manual_seed(len(shape) * 7 + shape[0])
    x = torch.randn(*shape, generator=g).to(dtype)
    t = torch.randn(*shape, generator=g).to(dtype)
    w = {"none": None, "rand": torch.rand(shape[0], generator=g).to(dtype),
         "tiny_negative": -torch.rand(shape[0], generator=g).to(dtype) * 1e-20}[weight]
    assert MOD._cpu_mse_ok(x, t, w)
    got = mean_squared_error(x, t, sample_weight=w, multioutput=mo)
    monkeypatch.setattr(MOD, "_cpu_mse_ok", lambda *a: False)
    want = mean_squared_error(x, t, sample_weight=w, multioutput=mo)
    assert got.dtype == want.dtype and got.shape == want.shape
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-12, equal_nan=True)


def test_mixed_dtypes_and_errors_keep_aten_path():
    x = torch.rand(4)
    assert not MOD._cpu_mse_ok(x, x.double(), None)
    with pytest.raises(ValueError):
        mean_squared_error(torch.rand(3), torch.rand(4))
