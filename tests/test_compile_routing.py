"""Under torch.compile the ops wrappers call the dispatcher ops (torch.ops.torcheval_amd.*) with
the schema's argument order; exercised here with Meta tensors (schema binding + Meta kernels) by
forcing the wrappers' compiling() test, so an arity / type mismatch shows up without a GPU."""
import pytest
import torch

import torcheval_amd.ops as ops
from torcheval_amd.ops import classification as C
from torcheval_amd.ops import reductions as R
from torcheval_amd.ops import rowsums as RS

pytestmark = pytest.mark.skipif(not ops.native_loaded(), reason="extension not built")
META = torch.device("meta")


@pytest.fixture
def compiling(monkeypatch):
    for mod in (R, C, ops):
        monkeypatch.setattr(mod, "compiling", lambda: True)


def test_column_moments_routes(compiling):
    x = torch.empty(16, 4, device=META)
    t = torch.empty(16, 4, device=META)
    sse = torch.empty(4, device=META)
    sw = torch.empty((), device=META)
    R.column_moments(x, t, None, sse=sse, sw=sw)
    out = R.mse_fused(x, t, None, raw_values=True)
    assert out.shape == (4,) and out.device == META
    out = R.r2_fused(x, t, "uniform_average", 0)
    assert out.shape == () and out.device == META


def test_ne_sums_routes(compiling):
    x = torch.empty(32, device=META)
    t = torch.empty(32, device=META)
    out, flag = R.ne_sums(x, t, None, False)
    assert out.shape == (1, 3) and flag.shape == (1,)


def test_binary_and_multilabel_counts_route(compiling):
    x = torch.empty(32, device=META)
    t = torch.empty(32, dtype=torch.int64, device=META)
    s = torch.empty(1, device=META)
    C.binary_counts(x, t, threshold=0.5, tp=s, tn=s, total=s)
    xm = torch.empty(8, 5, device=META)
    tm = torch.empty(8, 5, dtype=torch.int64, device=META)
    c = torch.empty((), device=META)
    C.multilabel_counts(xm, tm, threshold=0.5, k=0, criteria="hamming", num_correct=c, num_total=c)


def test_row_sums_routes(compiling):
    x = torch.empty(32, device=META)
    o = torch.empty((), device=META)
    RS.update(x, None, None, 1.0, [o], [RS.code(0, 0)], 1)
