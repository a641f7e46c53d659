"""K3s sample-sort binary AUROC (csrc/kernels/samplesort.hip) against the FP64 CPU path.

Covers the fast path's ranges (32K..2M samples), heavy ties (equal-to-splitter buckets), NaN /
inf / signed zeros, fractional and integer target dtypes, degenerate rows, and an adversarial
row built against the deterministic stratified sampler so that one bucket holds almost every
sample (the oversized-bucket global-memory sort)."""
import numpy as np
import pytest
import torch

from torcheval_amd.metrics.functional import binary_auroc
from torcheval_amd.metrics.functional.classification._curve import binary_areas
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _cpu(x, t):
    return binary_areas(x.cpu(), t.cpu(), roc=True, pr=False)[0].item()


def _gpu(x, t):
    out = torch.empty(1, dtype=torch.float64, device=DEV)
    native().binary_auroc_samplesort(x.to(DEV).contiguous(), t.to(DEV).contiguous(), out)
    return out.item()


def _check(x, t, tol=1e-9):
    ref = _cpu(x, t)
    got = _gpu(x, t)
    assert abs(got - ref) <= tol, (got, ref)


@pytest.mark.parametrize("n", [1 << 15, 100_003, 1 << 20, 1_000_003, 1 << 21])
def test_uniform_sizes(n):
    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, generator=g)
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t)


def test_supported_range():
    assert native().samplesort_auc_ok(1 << 15) and native().samplesort_auc_ok(1 << 21)
    assert not native().samplesort_auc_ok((1 << 15) - 1) and not native().samplesort_auc_ok((1 << 21) + 1)


@pytest.mark.parametrize("levels", [1, 2, 7, 100, 3000])
def test_heavy_ties(levels):
    n = 1 << 20
    g = torch.Generator().manual_seed(levels)
    x = torch.randint(0, levels, (n,), generator=g).float() / levels
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t)


def _stable_singleton_oracle(x, t):
    """FP64 AUROC with the reference's group rule (`diff != 0` ends a group, so every NaN / +inf
    / -inf sample is its own group) over a STABLE descending sort.  The reference itself sorts
    with torch.sort(stable=False), so its value on such rows depends on the sort's tie order;
    K3a and K3s both keep source order."""
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
    tp_start = np.concatenate([[0.0], tp_end[:-1]])
    length = np.diff(np.concatenate([[-1], tails]))
    p = tp_end - tp_start
    area = float(np.sum((length - p) * (tp_start + p / 2)))
    P = ts.sum()
    return area / (P * (n - P))


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
    assert abs(_gpu(x, t) - _stable_singleton_oracle(x, t)) <= 1e-9
    if case == "zeros":  # no order-dependent groups: the reference's own value
        _check(x, t)


@pytest.mark.parametrize("dtype", [torch.float32, torch.int64, torch.int32, torch.uint8, torch.bool])
def test_target_dtypes(dtype):
    n = 200_000
    g = torch.Generator().manual_seed(11)
    x = torch.rand(n, generator=g)
    t = torch.randint(0, 2, (n,), generator=g).to(dtype)
    _check(x, t.to(torch.float32) if dtype == torch.bool else t)


def test_fractional_targets():
    n = 500_000
    g = torch.Generator().manual_seed(5)
    x = torch.rand(n, generator=g)
    t = torch.rand(n, generator=g)
    _check(x, t, tol=1e-7)


def test_degenerate_rows():
    n = 1 << 16
    x = torch.rand(n)
    assert _gpu(x, torch.zeros(n, dtype=torch.int64)) == 0.5
    assert _gpu(x, torch.ones(n, dtype=torch.int64)) == 0.5
    _check(torch.full((n,), 0.25), torch.randint(0, 2, (n,)))


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


def test_oversized_bucket():
    # every sampled position holds a score outside (0.4, 0.6); every other sample a distinct
    # score inside it -> one "between" bucket of ~n - S samples (global-memory sort)
    n = 1 << 16
    B = 32  # samplesort_auc_buckets(65536)
    g = torch.Generator().manual_seed(9)
    x = 0.4 + 0.2 * torch.rand(n, generator=g, dtype=torch.float64)
    x = x.float()
    pos = _sample_positions(n, 4 * B)
    x[pos] = torch.where(torch.rand(len(pos), generator=g) < 0.5, torch.tensor(0.1), torch.tensor(0.9))
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t)


def test_dispatch_matches_radix_path(monkeypatch):
    n = 1 << 20
    g = torch.Generator().manual_seed(1)
    x = torch.rand(n, generator=g).to(DEV)
    t = torch.randint(0, 2, (n,), generator=g).to(DEV)
    monkeypatch.setenv("TORCHEVAL_AMD_K3S", "1")
    fast = binary_auroc(x, t).item()
    monkeypatch.setenv("TORCHEVAL_AMD_K3S", "0")
    slow = binary_auroc(x, t).item()
    assert abs(fast - slow) <= 1e-9


def test_repeatable():
    n = 1 << 20
    g = torch.Generator().manual_seed(2)
    x = torch.rand(n, generator=g).to(DEV)
    t = torch.randint(0, 2, (n,), generator=g).to(DEV)
    vals = {binary_auroc(x, t).item() for _ in range(5)}
    assert len(vals) == 1
