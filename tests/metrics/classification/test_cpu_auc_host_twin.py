"""The small-batch CPU AUROC / AUPRC host twin (csrc/runtime/cpu_metrics.cpp cpu_binary_auc)
against the vectorised ATen form of _curve.py: ties, NaN / inf scores, weights, soft and
boolean targets, several rows, strided views, rows without positives or negatives."""
import pytest
import torch

from torcheval_amd.metrics.functional.classification import _curve
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="extension not built")


def _both(x, t, w=None, monkeypatch=None):
    got = _curve.binary_areas(x, t, w, roc=True, pr=True)
    monkeypatch.setattr(_curve, "_CPU_AUC_MAX", -1)
    want = _curve.binary_areas(x, t, w, roc=True, pr=True)
    monkeypatch.setattr(_curve, "_CPU_AUC_MAX", 1 << 16)
    return got, want


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("tdtype", [torch.int64, torch.int32, torch.bool, torch.uint8, torch.float32])
@pytest.mark.parametrize("weighted", [False, True])
def test_host_twin_matches_aten(monkeypatch, dtype, tdtype, weighted):
    g = torch.Generator().manual_seed(3)
    for rows, n in [(1, 1), (1, 8), (3, 37), (2, 1000)]:
        x = (torch.rand(rows, n, generator=g) * 10).round().to(dtype)  # many ties
        x[0, 0] = float("nan")
        if n > 3:
            x[0, 1] = float("inf")
            x[-1, 2] = float("nan")
        t = torch.randint(0, 2, (rows, n), generator=g).to(tdtype)
        w = torch.rand(rows, n, generator=g).to(dtype) if weighted else None
        (r1, p1), (r2, p2) = _both(x, t, w, monkeypatch)
        torch.testing.assert_close(r1, r2, rtol=1e-12, atol=1e-12)
        torch.testing.assert_close(p1, p2, rtol=1e-12, atol=1e-12)
        assert r1.dtype == torch.float64 and r1.shape == (rows,)


def test_host_twin_edge_rows(monkeypatch):
    x = torch.tensor([[0.1, 0.5, 0.5, 0.9], [0.3, 0.3, 0.3, 0.3], [1.0, 2.0, 3.0, 4.0]])
    t = torch.tensor([[0, 0, 0, 0], [1, 0, 1, 0], [1, 1, 1, 1]])
    (r1, p1), (r2, p2) = _both(x, t, None, monkeypatch)
    torch.testing.assert_close(r1, r2)
    torch.testing.assert_close(p1, p2)
    assert r1[0] == 0.5 and p1[0] == 0.0  # no positives
    assert r1[1] == 0.5  # one tie group
    # soft targets and a strided (transposed) view
    g = torch.Generator().manual_seed(9)
    xs = torch.rand(50, 4, generator=g).t()
    ts = torch.rand(50, 4, generator=g).t()
    (r1, p1), (r2, p2) = _both(xs, ts, None, monkeypatch)
    torch.testing.assert_close(r1, r2, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(p1, p2, rtol=1e-12, atol=1e-12)


def test_functional_and_class_use_it():
    from torcheval_amd.metrics import BinaryAUPRC, BinaryAUROC
    from torcheval_amd.metrics.functional import binary_auprc, binary_auroc, multiclass_auroc

    g = torch.Generator().manual_seed(1)
    x, t = torch.rand(8, generator=g), torch.randint(0, 2, (8,), generator=g)
    want = _curve.binary_areas(x, t, None, roc=True, pr=True)
    assert binary_auroc(x, t) == want[0][0]
    ap = binary_auprc(x, t)
    assert ap == want[1][0].to(ap.dtype)
    m = BinaryAUROC()
    m.update(x, t)
    assert m.compute() == want[0][0]
    m2 = BinaryAUPRC()
    m2.update(x, t)
    assert m2.compute() == want[1][0].to(m2.compute().dtype)
    xm = torch.rand(20, 3, generator=g)
    tm = torch.randint(0, 3, (20,), generator=g)
    assert multiclass_auroc(xm, tm, num_classes=3).shape == ()
