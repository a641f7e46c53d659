"""Host (CPU) twins of the K1 / K4 kernels (csrc/runtime/cpu_metrics.cpp) against the ATen
paths they replace for small CPU batches: exact counts on random shapes, NaN scores, scores
equal to a threshold, float targets and strided views."""

import torch

from torcheval_amd.ops import native, native_loaded
from torcheval_amd.ops.binned import _binned_counts_aten
from torcheval_amd.ops.classification import native_cls


def test_cpu_binned_counts_exact():
    assert native_loaded()
    g = torch.Generator().manual_seed(0)
    for trial in range(120):
        n = int(torch.randint(1, 60, (1,), generator=g))
        c = int(torch.randint(1, 9, (1,), generator=g))
        t_n = int(torch.randint(1, 30, (1,), generator=g))
        x = torch.rand(n, c, generator=g)
        thr = torch.rand(t_n, generator=g).sort().values
        if trial % 3 == 0:
            x[0, 0] = float("nan")
        if trial % 4 == 0 and n > 1:
            x[1, 0] = thr[t_n // 2]
        if trial % 5 == 0:
            x = x.double()
        if trial % 7 == 0:
            x = x.t().contiguous().t()
        mode = trial % 2
        t = torch.randint(0, c, (n,), generator=g) if mode else torch.randint(0, 2, (n, c), generator=g)
        if mode == 0 and trial % 6 == 0:
            t = t.float()
        exp = _binned_counts_aten(x, t, thr, mode)
        buf = torch.zeros(3, t_n, c)
        native().cpu_binned_counts(x, t, thr, mode, buf[0], buf[1], buf[2])
        for a, b in zip(buf, exp):
            assert torch.equal(a, b), trial


def test_cpu_cls_counts_matches_histograms():
    g = torch.Generator().manual_seed(1)
    for trial in range(60):
        n, c = int(torch.randint(1, 40, (1,), generator=g)), int(torch.randint(2, 9, (1,), generator=g))
        x = torch.rand(n, c, generator=g)
        if trial % 4 == 0:
            x[0, c - 1] = float("nan")
        if trial % 5 == 0:
            x = x.double()
        y = torch.randint(0, c, (n,), generator=g)
        assert native_cls(x, y, num_classes=c)
        buf = torch.zeros(5, c)
        cm = torch.zeros(c * c)
        native().cpu_cls_counts(x, y, 1, c, None, None, buf[0], buf[1], buf[2], cm, None, 0, None, None, buf[3])
        pred = x.argmax(dim=1)
        hit = pred == y
        ones = torch.ones(n)
        torch.testing.assert_close(buf[0], torch.zeros(c).scatter_add_(0, y[hit], ones[hit]))
        torch.testing.assert_close(buf[1], torch.zeros(c).scatter_add_(0, y, ones))
        torch.testing.assert_close(buf[2], torch.zeros(c).scatter_add_(0, pred, ones))
        torch.testing.assert_close(buf[3], torch.zeros(c).scatter_add_(0, pred[~hit], ones[~hit]))
        torch.testing.assert_close(cm, torch.bincount(y * c + pred, minlength=c * c).float())


def test_out_of_range_labels_keep_the_aten_path():
    x = torch.rand(4, 3)
    assert not native_cls(x, torch.tensor([0, 1, 3, 2]), num_classes=3)
    assert not native_cls(torch.tensor([0, 5, 1, 2]), torch.tensor([0, 1, 1, 2]), num_classes=3)
    assert native_cls(x, torch.tensor([0, 1, 2, 2]), num_classes=3)
