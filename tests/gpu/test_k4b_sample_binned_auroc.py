"""K4b (csrc/kernels/binned_auroc.hip): the reference-default multiclass binned AUROC, one
value per sample (reference binned_auroc.py:189-215), against the ATen per-sample form on CPU
(`_per_sample_binned_auroc`, itself pinned to the reference's fixtures) on ties, NaN, duplicate
thresholds, T = 200, C from 2 to 1000, int32 / int64 labels and strided rows; out-of-range labels
raise the reference's error after one device-flag read."""

import pytest
import torch

from torcheval_amd.metrics import MulticlassBinnedAUROC
from torcheval_amd.metrics.functional import multiclass_binned_auroc
from torcheval_amd.metrics.functional.classification.binned_auroc import _per_sample_binned_auroc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _case(n, c, t, seed, ties=False, nan=False, dup_thr=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, c, generator=g)
    if ties:
        x = (x * 8).round() / 8
    if nan:
        x[torch.rand(n, c, generator=g) < 0.05] = float("nan")
    thr = torch.sort(torch.rand(t, generator=g))[0]
    if dup_thr:
        thr = torch.sort((thr * 4).round() / 4)[0]
    y = torch.randint(0, c, (n,), generator=g)
    return x, y, thr


@pytest.mark.parametrize("c", [2, 3, 4, 5, 17, 100, 257, 1000])
@pytest.mark.parametrize("kind", ["plain", "ties", "nan", "dup_thr"])
def test_matches_aten_per_sample(c, kind):
    x, y, thr = _case(3001, c, 200 if kind == "plain" else 13, c * 7 + len(kind),
                      ties=kind == "ties", nan=kind == "nan", dup_thr=kind == "dup_thr")
    ref = _per_sample_binned_auroc(x, y, c, thr)
    got, thr_out = multiclass_binned_auroc(x.to(DEV), y.to(DEV), num_classes=c, threshold=thr.to(DEV), average=None)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=1e-6)
    assert thr_out.device.type == "cuda"
    mac, _ = multiclass_binned_auroc(x.to(DEV), y.to(DEV), num_classes=c, threshold=thr.to(DEV))
    assert float(mac) == pytest.approx(float(ref.mean()), abs=1e-6)


def test_int32_labels_strided_rows_and_default_thresholds():
    g = torch.Generator().manual_seed(5)
    big = torch.rand(2000, 120, generator=g)
    x = big[:, 3:103]  # row stride 120, 4-B offset 3
    y = torch.randint(0, 100, (2000,), generator=g)
    ref = _per_sample_binned_auroc(x, y, 100, torch.linspace(0, 1, 200))
    got, _ = multiclass_binned_auroc(x.to(DEV), y.to(torch.int32).to(DEV), num_classes=100, threshold=200,
                                     average=None)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=1e-6)


def test_reference_fixture_on_gpu():
    x = torch.tensor([[0.1, 0.2, 0.1], [0.4, 0.2, 0.1], [0.6, 0.1, 0.2], [0.4, 0.2, 0.3], [0.6, 0.2, 0.4]])
    y = torch.tensor([0, 1, 2, 1, 0])
    v, _ = multiclass_binned_auroc(x.to(DEV), y.to(DEV), num_classes=3, threshold=5)
    assert float(v) == pytest.approx(0.4, abs=1e-7)
    r, _ = multiclass_binned_auroc(x.to(DEV), y.to(DEV), num_classes=3, threshold=5, average=None)
    torch.testing.assert_close(r.cpu(), torch.tensor([0.5, 0.25, 0.25, 0.0, 1.0]))


def test_bad_labels_raise_and_class_metric():
    x, y, thr = _case(500, 10, 20, 1)
    bad = y.clone()
    bad[7] = 10
    with pytest.raises(RuntimeError, match="Class values must be smaller than num_classes"):
        multiclass_binned_auroc(x.to(DEV), bad.to(DEV), num_classes=10, threshold=thr.to(DEV))
    bad[7] = -1
    with pytest.raises(RuntimeError, match="Class values must be smaller than num_classes"):
        multiclass_binned_auroc(x.to(DEV), bad.to(DEV), num_classes=10, threshold=thr.to(DEV))
    m = MulticlassBinnedAUROC(num_classes=10, threshold=thr.to(DEV), device=DEV)
    m.update(x[:200].to(DEV), y[:200].to(DEV))
    m.update(x[200:].to(DEV), y[200:].to(DEV))
    ref = _per_sample_binned_auroc(x, y, 10, thr).mean()
    assert float(m.compute()[0]) == pytest.approx(float(ref), abs=1e-6)


@pytest.mark.parametrize("t,c", [(5000, 7), (4096, 3), (4097, 64), (1, 5)])
def test_threshold_counts_past_the_lds_stage(t, c):
    """T > 4096 searches the thresholds in global memory instead of LDS; T = 1 and T = 4096 are
    the edges of the staged path."""
    x, y, thr = _case(1500, c, t, t + c)
    ref = _per_sample_binned_auroc(x, y, c, thr)
    got, _ = multiclass_binned_auroc(x.to(DEV), y.to(DEV), num_classes=c, threshold=thr.to(DEV), average=None)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=1e-6)
