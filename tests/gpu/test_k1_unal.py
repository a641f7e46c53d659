"""K1 on f32 rows of any width and alignment (the UNAL instantiations of classification.hip:
16-B loads at 4-B alignment, the row's last 4 columns rotated into place for the lane that
straddles the row end).  Widths 33..2050 that are not multiples of 4, rows starting at every
4-B phase (column-sliced views), adversarial ties / NaN / inf rows, against torch.argmax /
ATen counts on CPU (reference accuracy.py:260-278, precision.py:115-139, confusion_matrix.py:219-234)."""

import pytest
import torch

from torcheval_amd.metrics import (
    MulticlassAccuracy,
    MulticlassConfusionMatrix,
    MulticlassF1Score,
    MulticlassPrecision,
)
from torcheval_amd.metrics.functional import multiclass_accuracy

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rows(n, c, off, seed):
    g = torch.Generator().manual_seed(seed)
    big = torch.randn(n, c + 7, generator=g)
    x = big[:, off : off + c]
    y = torch.randint(0, c, (n,), generator=g)
    r = torch.arange(n)
    hit = torch.rand(n, generator=g) < 0.5
    x[hit, y[hit]] = 9.0
    last = r % 5 == 0
    y[last] = c - 1  # targets in the straddling lane's columns
    x[last, c - 1] = 9.0
    tb = (r % 7 == 0) & (y > 0)
    x[tb, 0] = x[tb, y[tb]]  # an earlier tie: wrong
    te = r % 11 == 0
    x[te, c - 1] = x[te, y[te]]  # a tie in the last column: still right unless it is the target
    x[r % 13 == 0, c - 2] = float("nan")
    x[r % 17 == 0, c - 1] = float("inf")
    return x, y


@pytest.mark.parametrize("c", [33, 257, 1001, 1002, 1003, 1023, 2050])
@pytest.mark.parametrize("off", [0, 1, 2, 3])
def test_micro_accuracy_odd(c, off):
    x, y = _rows(3000, c, off, c * 4 + off)
    want = float((x.argmax(1) == y).sum())
    m = MulticlassAccuracy(device=DEV)
    m.update(x.to(DEV), y.to(DEV))
    m.update(x.to(DEV), y.to(DEV))
    assert float(m.num_correct) == 2 * want and float(m.num_total) == 2 * x.shape[0]
    got = multiclass_accuracy(x.to(DEV), y.to(DEV))
    assert float(got) == pytest.approx(want / x.shape[0], abs=1e-7)


@pytest.mark.parametrize("c", [35, 1001, 2051])
@pytest.mark.parametrize("off", [1, 3])
def test_macro_topk_precision_confusion_odd(c, off):
    x, y = _rows(2000, c, off, c + off)
    xd, yd = x.to(DEV), y.to(DEV)
    ref_pred = x.argmax(1)
    # macro accuracy: per-class correct / label counts
    m = MulticlassAccuracy(average="macro", num_classes=c, device=DEV)
    m.update(xd, yd)
    corr = torch.zeros(c).index_add_(0, y, (ref_pred == y).float())
    lab = torch.zeros(c).index_add_(0, y, torch.ones(len(y)))
    torch.testing.assert_close(m.num_correct.cpu(), corr)
    torch.testing.assert_close(m.num_total.cpu(), lab)
    # top-k: rank of the target (strictly larger scores) < k
    k = 3
    mk = MulticlassAccuracy(k=k, device=DEV)
    mk.update(xd, yd)
    xt = x.gather(1, y[:, None])
    want_k = float(((x > xt).sum(1) < k).sum())
    assert float(mk.num_correct) == want_k
    # precision (predicted-label histograms) and the confusion matrix
    p = MulticlassPrecision(num_classes=c, average=None, device=DEV)
    p.update(xd, yd)
    tp = torch.zeros(c).index_add_(0, y, (ref_pred == y).float())
    fp = torch.zeros(c).index_add_(0, ref_pred, (ref_pred != y).float())
    torch.testing.assert_close(p.num_tp.cpu(), tp)
    torch.testing.assert_close(p.num_fp.cpu(), fp)
    cm = MulticlassConfusionMatrix(c, device=DEV)
    cm.update(xd, yd)
    ref_cm = torch.zeros(c, c).index_put_((y, ref_pred), torch.ones(len(y)), accumulate=True)
    torch.testing.assert_close(cm.confusion_matrix.cpu().float(), ref_cm)
    f1 = MulticlassF1Score(num_classes=c, average="macro", device=DEV)
    f1.update(xd, yd)
    f1c = MulticlassF1Score(num_classes=c, average="macro")
    f1c.update(x, y)
    torch.testing.assert_close(f1.compute().cpu(), f1c.compute())
