"""K3b bucketed binary AUROC / AUPRC (csrc/kernels/bucketauc.hip) against the FP64 CPU path.

Covers the supported range (32K..2M samples), heavy ties (equal-to-splitter bins), NaN / inf /
signed zeros (singleton groups in source order), fractional and integer target dtypes,
degenerate rows, and rows built against the deterministic stratified sampler so that one
"between" bin holds almost every sample: with distinct keys (multi-level sub-binning over the
global scratch), with a few repeated keys (the one-key closed form), and in LDS."""
import numpy as np
import pytest
import torch

from torcheval_amd.metrics.functional import binary_auprc, binary_auroc
from torcheval_amd.metrics.functional.classification._curve import binary_areas
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _cpu(x, t):
    r, p = binary_areas(x.cpu(), t.cpu(), roc=True, pr=True)
    return r.item(), p.item()


def _gpu(x, t, roc=True, pr=True):
    o_r = torch.full((1,), -7.0, dtype=torch.float64, device=DEV) if roc else None
    o_p = torch.full((1,), -7.0, dtype=torch.float64, device=DEV) if pr else None
    native().binary_auc_bucket(x.to(DEV).contiguous(), t.to(DEV).contiguous(), o_r, o_p)
    return (o_r.item() if roc else None), (o_p.item() if pr else None)


def _check(x, t, tol=1e-9):
    want = _cpu(x, t)
    got = _gpu(x, t)
    assert abs(got[0] - want[0]) <= tol, ("auroc", got, want)
    assert abs(got[1] - want[1]) <= tol, ("auprc", got, want)


@pytest.mark.parametrize("n", [1 << 15, 100_003, 1 << 20, 1_000_003, 1 << 21])
def test_uniform_sizes(n):
    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, generator=g)
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t)


def test_supported_range():
    assert native().bucket_auc_ok(1 << 15) and native().bucket_auc_ok(1 << 21)
    assert not native().bucket_auc_ok((1 << 15) - 1) and not native().bucket_auc_ok((1 << 21) + 1)


@pytest.mark.parametrize("levels", [1, 2, 7, 100, 3000, 100_000])
def test_heavy_ties(levels):
    n = 1 << 20
    g = torch.Generator().manual_seed(levels)
    x = torch.randint(0, levels, (n,), generator=g).float() / levels
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t)


def test_normal_scores_and_imbalance():
    n = 750_000
    g = torch.Generator().manual_seed(4)
    t = (torch.rand(n, generator=g) < 0.03).long()
    x = torch.randn(n, generator=g) + 1.5 * t
    _check(x, t)


def _stable_singleton_oracle(x, t):
    """FP64 (AUROC, AUPRC) with the reference's group rule (`diff != 0` ends a group, so every
    NaN / +inf / -inf sample is its own group) over a STABLE descending sort.  The reference
    itself sorts with torch.sort(stable=False), so its value on such rows depends on the sort's
    tie order; K3a and K3b both keep source order."""
    xs = x.double().numpy()
    ts = t.double().numpy()
    n = len(xs)
    cls = np.where(np.isnan(xs), 0, np.where(xs == np.inf, 1, np.where(xs == -np.inf, 3, 2)))
    fin = np.where(cls == 2, xs, 0.0)
    order = np.lexsort((np.arange(n), -fin, cls))
    s, tt, c = fin[order], ts[order], cls[order]
    same_next = (c[:-1] == 2) & (c[1:] == 2) & (s[:-1] == s[1:])
    tails = np.flatnonzero(np.append(~same_next, True))
    tp_end = np.cumsum(tt)[tails]
    cnt_end = (tails + 1).astype(np.float64)
    tp_start = np.concatenate([[0.0], tp_end[:-1]])
    length = np.diff(np.concatenate([[-1], tails]))
    p = tp_end - tp_start
    P = ts.sum()
    roc = float(np.sum((length - p) * (tp_start + p / 2))) / (P * (n - P))
    pr = float(np.sum(p * tp_end / cnt_end)) / P
    return roc, pr


@pytest.mark.parametrize("case", ["nan", "pinf", "ninf", "zeros", "mixed"])
def test_special_values(case):
    n = 300_000
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, generator=g)
    idx = torch.randperm(n, generator=g)
    if case in ("nan", "mixed"):
        x[idx[:500]] = float("nan")
    if case in ("pinf", "mixed"):
        x[idx[500:900]] = float("inf")
    if case in ("ninf", "mixed"):
        x[idx[900:1300]] = float("-inf")
    if case in ("zeros", "mixed"):
        x[idx[1300:5000]] = 0.0
        x[idx[5000:9000]] = -0.0
    t = torch.randint(0, 2, (n,), generator=g)
    want = _stable_singleton_oracle(x, t)
    got = _gpu(x, t)
    assert abs(got[0] - want[0]) <= 1e-9 and abs(got[1] - want[1]) <= 1e-9, (got, want)
    if case == "zeros":  # no order-dependent groups: the reference's own value
        _check(x, t)


@pytest.mark.parametrize("dtype", [torch.float32, torch.int64, torch.int32, torch.uint8, torch.bool])
def test_target_dtypes(dtype):
    n = 200_000
    g = torch.Generator().manual_seed(11)
    x = torch.rand(n, generator=g)
    t = torch.randint(0, 2, (n,), generator=g).to(dtype)
    want = _cpu(x, t.to(torch.float32))
    got = _gpu(x, t)
    assert abs(got[0] - want[0]) <= 1e-9 and abs(got[1] - want[1]) <= 1e-9


def test_fractional_targets():
    n = 500_000
    g = torch.Generator().manual_seed(5)
    x = torch.rand(n, generator=g)
    t = torch.rand(n, generator=g)
    _check(x, t, tol=1e-7)


def test_degenerate_rows():
    n = 1 << 16
    x = torch.rand(n)
    for t in (torch.zeros(n, dtype=torch.int64), torch.ones(n, dtype=torch.int64)):
        want = _cpu(x, t)
        got = _gpu(x, t)
        assert got[0] == 0.5 and abs(got[1] - want[1]) <= 1e-12, (got, want)
    _check(torch.full((n,), 0.25), torch.randint(0, 2, (n,)))


def test_one_output_only():
    n = 1 << 17
    g = torch.Generator().manual_seed(8)
    x, t = torch.rand(n, generator=g), torch.randint(0, 2, (n,), generator=g)
    want = _cpu(x, t)
    assert abs(_gpu(x, t, pr=False)[0] - want[0]) <= 1e-9
    assert abs(_gpu(x, t, roc=False)[1] - want[1]) <= 1e-9


def _buckets(n):
    b = 16
    while b < 1024 and b * 1024 < n:
        b *= 2
    return b


def _sample_positions(n, S):
    q = n // S
    pos = []
    for s in range(S):
        h = (s * 2654435761) & 0xFFFFFFFF
        h ^= h >> 15
        h = (h * 2246822519) & 0xFFFFFFFF
        h ^= h >> 13
        pos.append(s * q + h % q)
    return torch.tensor(pos)


def _oversized(n, inside, seed):
    """Every sampled position holds 0.1 or 0.9, every other sample `inside` (in (0.4, 0.6)):
    one between bin of ~n - S samples."""
    g = torch.Generator().manual_seed(seed)
    x = inside(n, g)
    pos = _sample_positions(n, 4 * _buckets(n))
    x[pos] = torch.where(torch.rand(len(pos), generator=g) < 0.5, torch.tensor(0.1), torch.tensor(0.9))
    return x, torch.randint(0, 2, (n,), generator=g)


def test_oversized_bin_distinct_keys():
    # 65536 samples: global scratch, span ~2^23 ulps -> pushed sub-bins, two more levels
    _check(*_oversized(1 << 16, lambda n, g: (0.4 + 0.2 * torch.rand(n, generator=g, dtype=torch.float64)).float(), 9))


def test_oversized_bin_dense_keys():
    # 1M distinct consecutive floats just above 0.5: ~2^20 ulps, every sub-bin of level 0 pushed
    def inside(n, g):
        return (0.5 + torch.randperm(n, generator=g).double() * 2.0**-24).float()

    _check(*_oversized(1 << 20, inside, 10))


def test_oversized_bin_few_keys():
    # 100 repeated keys inside the bin: sub-bins of one key resolved in closed form
    def inside(n, g):
        return 0.45 + 0.1 * torch.randint(0, 100, (n,), generator=g).float() / 100

    _check(*_oversized(1 << 18, inside, 12))


def test_bin_fits_lds():
    # ~3000 samples in one between bin: the LDS-staged path with a pushed level
    n = 1 << 15
    g = torch.Generator().manual_seed(13)
    x = torch.rand(n, generator=g)
    pos = _sample_positions(n, 4 * _buckets(n))
    keep = torch.ones(n, dtype=torch.bool)
    keep[pos] = False
    inner = keep.nonzero().flatten()[:3000]
    x[inner] = 0.5 + torch.arange(3000).float() * 2.0**-24
    _check(x, torch.randint(0, 2, (n,), generator=g))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_dispatch_matches_radix_path(monkeypatch, dtype):
    n = 1 << 20
    g = torch.Generator().manual_seed(1)
    x = torch.rand(n, generator=g).to(dtype).to(DEV)
    t = torch.randint(0, 2, (n,), generator=g).to(DEV)
    monkeypatch.setenv("TORCHEVAL_AMD_K3B", "1")
    fast = (binary_auroc(x, t).item(), binary_auprc(x, t).item())
    monkeypatch.setenv("TORCHEVAL_AMD_K3B", "0")
    slow = (binary_auroc(x, t).item(), binary_auprc(x, t).item())
    assert abs(fast[0] - slow[0]) <= 1e-9 and abs(fast[1] - slow[1]) <= 1e-9


def test_repeatable():
    n = 1 << 20
    g = torch.Generator().manual_seed(2)
    x = torch.rand(n, generator=g).to(DEV)
    t = torch.randint(0, 2, (n,), generator=g).to(DEV)
    vals = {(binary_auroc(x, t).item(), binary_auprc(x, t).item()) for _ in range(5)}
    assert len(vals) == 1
