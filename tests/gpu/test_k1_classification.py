"""K1 fused classification kernel vs a plain-PyTorch fp32 reference (MI355X only)."""

import pytest
import torch

from torcheval_amd.ops import native_loaded
from torcheval_amd.ops.classification import binary_counts, cls_counts

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_argmax(x: torch.Tensor) -> torch.Tensor:
    # fp32 CPU reference with torch.argmax semantics (first max, NaN is max)
    return x.float().cpu().argmax(dim=1)


def test_native_loaded():
    assert native_loaded()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,c", [(1, 1), (5, 3), (257, 7), (8192, 1000), (300, 1024), (64, 4097)])
def test_micro_and_histograms(dtype, n, c):
    g = torch.Generator().manual_seed(n * 31 + c)
    x = torch.randn(n, c, generator=g).to(dtype)
    y = torch.randint(0, c, (n,), generator=g)
    xd, yd = x.to(DEV), y.to(DEV)
    pred = _ref_argmax(x)
    correct = (pred == y)
    out = torch.zeros(2, device=DEV)
    cc = torch.zeros(c, device=DEV)
    cl = torch.zeros(c, device=DEV)
    cp = torch.zeros(c, device=DEV)
    cm = torch.zeros(c * c, device=DEV)
    cls_counts(xd, yd, k=1, num_classes=c, micro_correct=out[0:1], micro_total=out[1:2],
               cls_correct=cc, cls_label=cl, cls_pred=cp, confusion=cm)
    torch.cuda.synchronize()
    assert out[0].item() == correct.sum().item()
    assert out[1].item() == n
    torch.testing.assert_close(cc.cpu(), torch.zeros(c).index_add_(0, y, correct.float()))
    torch.testing.assert_close(cl.cpu(), torch.bincount(y, minlength=c).float())
    torch.testing.assert_close(cp.cpu(), torch.bincount(pred, minlength=c).float())
    ref_cm = torch.zeros(c * c).index_add_(0, y * c + pred, torch.ones(n))
    torch.testing.assert_close(cm.cpu(), ref_cm)


@pytest.mark.parametrize("k", [2, 5])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_topk(k, dtype):
    g = torch.Generator().manual_seed(k)
    n, c = 4099, 130
    x = torch.randn(n, c, generator=g).to(dtype)
    y = torch.randint(0, c, (n,), generator=g)
    xf = x.float()
    rank = (xf > xf.gather(1, y[:, None])).sum(1)
    expected = (rank < k).sum().item()
    out = torch.zeros(2, device=DEV)
    cls_counts(x.to(DEV), y.to(DEV), k=k, num_classes=c, micro_correct=out[0:1], micro_total=out[1:2])
    assert out[0].item() == expected


def test_ties_nan_and_inf():
    x = torch.tensor([
        [1.0, 3.0, 3.0, 0.0],
        [float("nan"), 5.0, float("nan"), 1.0],
        [-float("inf")] * 4,
        [0.0, float("inf"), float("inf"), 2.0],
    ])
    y = torch.tensor([1, 0, 0, 2])
    cp = torch.zeros(4, device=DEV)
    out = torch.zeros(2, device=DEV)
    cls_counts(x.to(DEV), y.to(DEV), num_classes=4, micro_correct=out[0:1], cls_pred=cp)
    pred = x.argmax(1)
    torch.testing.assert_close(cp.cpu(), torch.bincount(pred, minlength=4).float())
    assert out[0].item() == (pred == y).sum().item()


def test_noncontiguous_and_int32_targets():
    x = torch.randn(1000, 64)
    xt = x.t().contiguous().t()  # column-major view
    y = torch.randint(0, 64, (1000,), dtype=torch.int32)
    out = torch.zeros(1, device=DEV)
    cls_counts(xt.to(DEV), y.to(DEV), num_classes=64, micro_correct=out)
    assert out.item() == (x.argmax(1) == y.long()).sum().item()
    xs = torch.randn(500, 130)[:, :100]  # row stride 130 (not 16-B aligned rows)
    ys = torch.randint(0, 100, (500,))
    out.zero_()
    cls_counts(xs.to(DEV), ys.to(DEV), num_classes=100, micro_correct=out)
    assert out.item() == (xs.argmax(1) == ys).sum().item()


def test_label_inputs_and_bad_targets():
    p = torch.randint(0, 10, (10000,))
    y = torch.randint(0, 10, (10000,))
    y[17] = 11  # out of range
    cl = torch.zeros(10, device=DEV)
    out = torch.zeros(1, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    cls_counts(p.to(DEV), y.to(DEV), num_classes=10, micro_correct=out, cls_label=cl, err=err)
    assert out.item() == (p == y).sum().item()
    valid = y[y < 10]
    torch.testing.assert_close(cl.cpu(), torch.bincount(valid, minlength=10).float())
    assert err.item() & 1


@pytest.mark.parametrize("tdtype", [torch.int64, torch.float32, torch.bool])
def test_binary_counts(tdtype):
    g = torch.Generator().manual_seed(7)
    x = torch.rand(100003, generator=g)
    t = torch.randint(0, 2, (100003,), generator=g).to(tdtype)
    w = torch.rand(100003, generator=g)
    buf = torch.zeros(5, device=DEV)
    binary_counts(x.to(DEV), t.to(DEV), threshold=0.3, weight=w.to(DEV), tp=buf[0:1], fp=buf[1:2],
                  tn=buf[2:3], fn=buf[3:4], total=buf[4:5])
    p = (x >= 0.3)
    tb = t.bool() if tdtype != torch.float32 else t == 1
    ref = torch.stack([(w * (p & tb)).sum(), (w * (p & ~tb)).sum(), (w * (~p & ~tb)).sum(),
                       (w * (~p & tb)).sum(), torch.tensor(100003.0)])
    torch.testing.assert_close(buf.cpu(), ref, rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("n,c", [(8192, 1000), (100000, 64), (3, 1000), (70000, 33), (5000, 10)])
def test_micro_fold_accumulates_exactly(n, c):
    # many back-to-back launches sharing the per-stream fold workspace must count exactly
    g = torch.Generator().manual_seed(n + c)
    x = torch.randn(n, c, generator=g)
    y = torch.randint(0, c, (n,), generator=g)
    x[:, 0] = torch.where(torch.rand(n, generator=g) < 0.3, 100.0, x[:, 0])  # many correct rows
    exp = (x.argmax(1) == y).sum().item()
    out = torch.zeros(2, device=DEV)
    xd, yd = x.to(DEV), y.to(DEV)
    for _ in range(25):
        cls_counts(xd, yd, num_classes=c, micro_correct=out[0:1], micro_total=out[1:2])
    torch.cuda.synchronize()
    assert out[0].item() == 25 * exp
    assert out[1].item() == 25 * n


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("c", [33, 1000, 1024, 1025, 2048])
def test_pred_free_accuracy_path(dtype, c):
    """micro / macro accuracy need no predicted label: the kernel first compares the row max
    with the target's score and only locates the argmax on a tie with it.  Rows here are ~85%
    correct, with exact ties before / after the target, NaN, +-inf and -0 / +0."""
    g = torch.Generator().manual_seed(c)
    n = 6000
    x = torch.randn(n, c, generator=g)
    y = torch.randint(0, c, (n,), generator=g)
    hit = torch.rand(n, generator=g) < 0.85
    x[hit, y[hit]] = 10.0  # target is the max
    r = torch.arange(n)
    tie_before = r % 7 == 0
    x[tie_before & (y > 0), 0] = x[tie_before & (y > 0), y[tie_before & (y > 0)]]  # earlier tie -> wrong
    tie_after = r % 11 == 0
    last = torch.full((n,), c - 1)
    x[tie_after, last[tie_after]] = x[tie_after, y[tie_after]]  # later tie -> still right
    x[r % 13 == 0, c // 2] = float("nan")
    x[r % 17 == 0, 1] = float("inf")
    z = r % 19 == 0
    x[z] = 0.0
    x[z, 0] = -0.0  # -0 and +0 tie: first index wins
    x = x.to(dtype)
    pred = _ref_argmax(x)
    correct = pred == y
    out = torch.zeros(2, device=DEV)
    cc = torch.zeros(c, device=DEV)
    cl = torch.zeros(c, device=DEV)
    cls_counts(x.to(DEV), y.to(DEV), k=1, num_classes=c, micro_correct=out[0:1], micro_total=out[1:2],
               cls_correct=cc, cls_label=cl)
    torch.cuda.synchronize()
    assert out[0].item() == correct.sum().item()
    torch.testing.assert_close(cc.cpu(), torch.zeros(c).index_add_(0, y, correct.float()))
    torch.testing.assert_close(cl.cpu(), torch.bincount(y, minlength=c).float())
