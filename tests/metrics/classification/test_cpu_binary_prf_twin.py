"""The small-batch CPU host twin of binary precision / recall / F1 (cpu_metrics.cpp cpu_binary_prf)
against the ATen forms of the same functions: value, dtype and warnings, over thresholds, NaN
inputs, every integer / bool target dtype, targets outside {0, 1}, empty batches and the
no-positive / no-prediction corners."""
import logging

import pytest
import torch

from torcheval_amd.metrics.functional import binary_f1_score, binary_precision, binary_recall
from torcheval_amd.metrics.functional.classification import f1_score as F1
from torcheval_amd.metrics.functional.classification import precision as P
from torcheval_amd.metrics.functional.classification import recall as R
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="extension not built")

FNS = [(binary_precision, P), (binary_recall, R), (binary_f1_score, F1)]


def _aten(fn, mod, monkeypatch, *args, **kw):
    monkeypatch.setattr(mod, "_cpu_prf_ok", lambda *a: False)
    try:
        return fn(*args, **kw)
    finally:
        monkeypatch.undo()


def _cases():
    g = torch.Generator().manual_seed(4)
    x = torch.rand(41, generator=g)
    x[3] = float("nan")
    x[7] = 0.5
    yield x, torch.randint(0, 2, (41,), generator=g)
    yield x.double(), torch.randint(0, 2, (41,), generator=g).bool()
    yield x, torch.randint(0, 2, (41,), generator=g).to(torch.int32)
    yield x, torch.randint(0, 2, (41,), generator=g).to(torch.uint8)
    yield x, torch.randint(0, 3, (41,), generator=g)  # a 2 counts 2 in sums, 0 in pred & target
    yield x, torch.zeros(41, dtype=torch.int64)  # no positives
    yield torch.zeros(41), torch.randint(0, 2, (41,), generator=g)  # no predictions above 0.5? (0 < 0.5)
    yield torch.ones(41), torch.ones(41, dtype=torch.int64)
    yield torch.zeros(0), torch.zeros(0, dtype=torch.int64)


@pytest.mark.parametrize("thr", [0.5, 0.0, 0.25])
@pytest.mark.parametrize("k", range(3))
def test_twin_matches_aten(monkeypatch, caplog, thr, k):
    fn, mod = FNS[k]
    for x, t in _cases():
        assert P._cpu_prf_ok(x, t)
        with caplog.at_level(logging.WARNING):
            caplog.clear()
            got = fn(x, t, threshold=thr)
            got_logs = [r.getMessage() for r in caplog.records]
            caplog.clear()
            want = _aten(fn, mod, monkeypatch, x, t, threshold=thr)
            want_logs = [r.getMessage() for r in caplog.records]
        assert got.dtype == want.dtype and got.shape == want.shape
        assert torch.equal(got, want) or (got.isnan() and want.isnan()), (fn.__name__, x, t, got, want)
        assert got_logs == want_logs


def test_float_targets_and_errors_keep_aten_path():
    x = torch.rand(5)
    assert not P._cpu_prf_ok(x, torch.rand(5))
    with pytest.raises(ValueError):
        binary_precision(torch.rand(3), torch.randint(0, 2, (4,)))
    with pytest.raises(ValueError):
        binary_recall(torch.rand(2, 2), torch.randint(0, 2, (2, 2)))


@pytest.mark.parametrize("cls_name,mod_name", [("BinaryPrecision", "precision"), ("BinaryRecall", "recall"),
                                               ("BinaryF1Score", "f1_score")])
def test_class_updates_match_aten(monkeypatch, cls_name, mod_name):
    import importlib

    import torcheval_amd.metrics as M

    mod = importlib.import_module(f"torcheval_amd.metrics.classification.{mod_name}")
    fast, slow = getattr(M, cls_name)(), getattr(M, cls_name)()
    batches = list(_cases())
    for x, t in batches:
        fast.update(x, t)
    monkeypatch.setattr(mod, "_cpu_prf_ok", lambda *a: False)
    for x, t in batches:
        slow.update(x, t)
    for name in fast._state_name_to_default:
        a, b = getattr(fast, name), getattr(slow, name)
        assert a.dtype == b.dtype and torch.equal(a, b), (name, a, b)
    torch.testing.assert_close(fast.compute(), slow.compute(), equal_nan=True)
