"""K5 v2 (one-launch column moments, reductions.hip moments_v2_kernel) at widths that are not
multiples of 4, at column offsets 1-3 (rows start at every 4-B phase), with and without row
weights, through every tile geometry (forced with TORCHEVAL_AMD_K5_CG / _BLOCKS / _MAXR), vs
fp64 CPU references of the same formulas (reference mean_squared_error.py:82-111,
r2_score.py:97-130)."""

import pytest
import torch

from torcheval_amd.metrics import MeanSquaredError, R2Score
from torcheval_amd.metrics.functional import mean_squared_error, r2_score

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _view(n, d, off, g, scale=1.0, shift=0.0):
    """[n, d] view whose rows start `off` floats into rows of width d + 5 (any 4-B phase)."""
    big = torch.randn(n, d + 5, generator=g) * scale + shift
    return big[:, off : off + d]


def _mse_ref(x, y, w=None):
    e = (y.double() - x.double()) ** 2
    if w is None:
        return e.sum(0), torch.tensor(float(x.shape[0]), dtype=torch.float64)
    w = w.double()
    return (e * w[:, None]).sum(0), w.sum()


@pytest.fixture(params=[(None, None, None), ("4", "64", None), ("16", "256", "4"), ("64", "1024", "2")],
                ids=["auto", "cg4", "cg16", "cg64"])
def geometry(request, monkeypatch):
    cg, blocks, maxr = request.param
    monkeypatch.setenv("TORCHEVAL_AMD_AB_DYNAMIC", "1")  # the native side re-reads the knobs per call
    for k, v in (("TORCHEVAL_AMD_K5_CG", cg), ("TORCHEVAL_AMD_K5_BLOCKS", blocks), ("TORCHEVAL_AMD_K5_MAXR", maxr)):
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, v)
    return request.param


@pytest.mark.parametrize("d", [4, 5, 7, 63, 65, 257, 1001])
@pytest.mark.parametrize("off", [0, 1, 3])
@pytest.mark.parametrize("weighted", [False, True])
def test_mse_class_odd_widths(geometry, d, off, weighted):
    g = torch.Generator().manual_seed(d * 7 + off)
    m = MeanSquaredError(multioutput="raw_values", device=DEV)
    xs, ys, ws = [], [], []
    for n in (1, 37, 3001):
        x, y = _view(n, d, off, g), _view(n, d, off, g)
        w = torch.rand(n, generator=g) if weighted else None
        m.update(x.to(DEV), y.to(DEV), sample_weight=None if w is None else w.to(DEV))
        xs.append(x)
        ys.append(y)
        ws.append(w)
    sse, sw = _mse_ref(torch.cat(xs), torch.cat(ys), torch.cat(ws) if weighted else None)
    torch.testing.assert_close(m.sum_squared_error.cpu().double(), sse, rtol=2e-6, atol=1e-5)
    torch.testing.assert_close(m.sum_weight.cpu().double(), sw, rtol=2e-6, atol=1e-5)
    torch.testing.assert_close(m.compute().cpu().double(), sse / sw, rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("d", [6, 1001, 4097])
@pytest.mark.parametrize("off", [1, 2])
@pytest.mark.parametrize("mo", ["uniform_average", "raw_values"])
@pytest.mark.parametrize("weighted", [False, True])
def test_mse_functional_odd_widths(geometry, d, off, mo, weighted):
    g = torch.Generator().manual_seed(d + off)
    x, y = _view(2049, d, off, g), _view(2049, d, off, g)
    w = torch.rand(2049, generator=g) if weighted else None
    ref = mean_squared_error(x.double(), y.double(), sample_weight=None if w is None else w.double(), multioutput=mo)
    got = mean_squared_error(x.to(DEV), y.to(DEV), sample_weight=None if w is None else w.to(DEV), multioutput=mo)
    assert got.shape == ref.shape
    torch.testing.assert_close(got.cpu().double(), ref, rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("d", [5, 1001])
@pytest.mark.parametrize("off", [0, 3])
@pytest.mark.parametrize("mo", ["uniform_average", "raw_values", "variance_weighted"])
@pytest.mark.parametrize("k", [0, 2])
def test_r2_odd_widths(geometry, d, off, mo, k):
    g = torch.Generator().manual_seed(3 * d + off)
    x, y = _view(1500, d, off, g), _view(1500, d, off, g, shift=2.0)
    ref = r2_score(x.double(), y.double(), multioutput=mo, num_regressors=k)
    got = r2_score(x.to(DEV), y.to(DEV), multioutput=mo, num_regressors=k)
    torch.testing.assert_close(got.cpu().double(), ref, rtol=1e-4, atol=1e-5)
    m = R2Score(multioutput=mo, num_regressors=k, device=DEV)
    for i in range(3):
        m.update(x[i::3].to(DEV), y[i::3].to(DEV))
    torch.testing.assert_close(m.compute().cpu().double(), ref, rtol=1e-4, atol=1e-5)


def test_nan_inf_rows_propagate(geometry):
    # a NaN in one column poisons only that column; clamped duplicate rows never leak values
    g = torch.Generator().manual_seed(1)
    x, y = _view(333, 9, 1, g), _view(333, 9, 1, g)
    x = x.clone()
    x[17, 2] = float("nan")
    x[300, 8] = float("inf")
    got = mean_squared_error(x.to(DEV), y.to(DEV), multioutput="raw_values").cpu()
    ref = mean_squared_error(x.double(), y.double(), multioutput="raw_values")
    assert torch.isnan(got[2]) and torch.isinf(got[8])
    keep = [0, 1, 3, 4, 5, 6, 7]
    torch.testing.assert_close(got[keep].double(), ref[keep], rtol=2e-5, atol=1e-6)


def test_deterministic_across_calls(geometry):
    g = torch.Generator().manual_seed(2)
    x, y = _view(8192, 1001, 1, g), _view(8192, 1001, 1, g)
    xd, yd = x.to(DEV), y.to(DEV)
    a = mean_squared_error(xd, yd, multioutput="raw_values")
    for _ in range(5):
        assert torch.equal(mean_squared_error(xd, yd, multioutput="raw_values"), a)
