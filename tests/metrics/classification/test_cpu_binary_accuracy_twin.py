"""The small-batch CPU host twin of binary accuracy (cpu_metrics.cpp) against the ATen form of
the reference's update (torch.where(input < threshold, 0, 1) == target)."""
import math

import pytest
import torch

from torcheval_amd.metrics import BinaryAccuracy
from torcheval_amd.metrics.functional import binary_accuracy
from torcheval_amd.metrics.functional.classification import accuracy as F_acc
from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="extension not built")


def _aten(x, t, thr):
    pred = torch.where(x < thr, 0, 1)
    return (pred == t).sum() / torch.tensor(t.shape[0])


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("tdtype", [torch.int64, torch.int32, torch.bool, torch.uint8, torch.float32, torch.float64])
@pytest.mark.parametrize("thr", [0.5, 0.0, 0.3000000001, 1.0])
def test_twin_matches_aten(dtype, tdtype, thr):
    g = torch.Generator().manual_seed(2)
    x = torch.rand(37, generator=g).to(dtype)
    x[3] = float("nan")
    x[5] = thr  # exactly at the threshold: predicted 1
    t = torch.randint(0, 2, (37,), generator=g).to(tdtype)
    assert F_acc._cpu_binary_ok(x, t)
    got = binary_accuracy(x, t, threshold=thr)
    want = _aten(x, t, thr)
    assert got.dtype == want.dtype and torch.equal(got, want)
    m = BinaryAccuracy(threshold=thr)
    m.update(x, t)
    m.update(x[:10], t[:10])
    want_c = ((torch.where(x < thr, 0, 1) == t).sum() + (torch.where(x[:10] < thr, 0, 1) == t[:10]).sum()).float()
    assert m.num_correct == want_c and m.num_total == 47.0
    assert m.compute() == want_c / 47


def test_twin_soft_targets_and_empty():
    x = torch.tensor([0.2, 0.7, 0.9])
    t = torch.tensor([0.5, 1.0, 0.0])  # 0.5 never equals a 0/1 prediction
    assert binary_accuracy(x, t) == _aten(x, t, 0.5)
    e = binary_accuracy(torch.zeros(0), torch.zeros(0))
    assert math.isnan(float(e))


def test_errors_still_raised():
    with pytest.raises(ValueError, match="same dimensions"):
        binary_accuracy(torch.rand(3), torch.rand(4))
    with pytest.raises(ValueError, match="one-dimensional"):
        BinaryAccuracy().update(torch.rand(2, 2), torch.rand(2, 2))
