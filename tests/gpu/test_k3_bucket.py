"""K3a splitter-bucket mode (csrc/kernels/radix.hip: a sorted 8192-key sample gives 255
splitters, ONE stable onesweep pass scatters the keys into 256 buckets, one workgroup per bucket
sorts it in LDS) against torch.sort(stable=True): continuous and clustered scores, tie-heavy rows
whose tie group exceeds a bucket's LDS capacity, NaN / +-0 / +-inf, payloads, ascending order,
and a row whose strided sample misrepresents it (buckets past the LDS capacity: the
single-workgroup LSD path)."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _bucket_mode(monkeypatch):
    # opt-in mode (read per sort): measured slower than the default onesweep passes at 1M
    monkeypatch.setenv("TORCHEVAL_AMD_K3_BUCKET", "1")


def _check(x: torch.Tensor, payload=None, kind: int = 0, ascending: bool = False) -> None:
    from torcheval_amd.ops import native

    xd = x.to(DEV)
    s = torch.empty_like(xd)
    idx = torch.empty(xd.shape, dtype=torch.int32, device=DEV)
    native().sort_desc(xd, s, idx, None if payload is None else payload.to(DEV), kind, None, ascending)
    ref_vals, ref_idx = torch.sort(x, dim=-1, descending=not ascending, stable=True)
    torch.testing.assert_close(s.cpu(), ref_vals, equal_nan=True, rtol=0, atol=0)
    got = idx.cpu().long()
    if kind == 0:
        assert torch.equal(got, ref_idx), "permutation differs from the stable reference"
    elif kind == 1:
        want = torch.gather(payload.float().expand(x.shape) if payload.dim() == 1 else payload.float(), 1, ref_idx)
        torch.testing.assert_close(idx.cpu().view(torch.float32), want, rtol=0, atol=0)
    else:
        want = torch.gather(payload.long().expand(x.shape) if payload.dim() == 1 else payload.long(), 1, ref_idx)
        assert torch.equal(got, want)


def _gen(kind: str, n: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    if kind == "uniform":
        return torch.rand(1, n, generator=g)
    if kind == "logits":
        return torch.randn(1, n, generator=g) * 3
    if kind == "sigmoid_confident":  # most scores crowd just below 1.0
        return torch.sigmoid(torch.randn(1, n, generator=g) * 3 + 6)
    if kind == "ties40":  # a 40% tie group: one bucket over the LDS capacity, tie run appended
        x = torch.rand(1, n, generator=g)
        x[:, torch.rand(n, generator=g) < 0.4] = 0.5
        return x
    if kind == "levels":
        return torch.randint(0, 7, (1, n), generator=g).float() / 7
    if kind == "special":
        x = torch.rand(1, n, generator=g) * 2 - 1
        m = torch.rand(n, generator=g)
        x[:, m < 0.01] = float("nan")
        x[:, (m >= 0.01) & (m < 0.02)] = -0.0
        x[:, (m >= 0.02) & (m < 0.03)] = 0.0
        x[:, (m >= 0.03) & (m < 0.035)] = float("inf")
        x[:, (m >= 0.035) & (m < 0.04)] = float("-inf")
        return x
    if kind == "constant":
        return torch.full((1, n), 0.25)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["uniform", "logits", "sigmoid_confident", "ties40", "levels", "special", "constant"])
@pytest.mark.parametrize("n", [65536, 1_000_000, 2_000_000])
def test_bucket_sort_matches_stable_sort(kind, n):
    _check(_gen(kind, n, n + len(kind)))


@pytest.mark.parametrize("n", [70_001, 1_000_000])
def test_payloads_and_ascending(n):
    g = torch.Generator().manual_seed(n)
    x = torch.rand(1, n, generator=g)
    x[:, ::97] = 0.5  # ties
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t, 1)
    _check(x, t.bool(), 1)
    _check(x, t.float(), 1)
    _check(x, torch.randint(0, 5, (1, n), generator=g), 2)
    _check(x, ascending=True)
    _check(_gen("special", n, 3), ascending=True)


def test_multi_row():
    g = torch.Generator().manual_seed(5)
    x = torch.rand(4, 300_000, generator=g)
    x[1] = (x[1] * 10).floor() / 10
    x[2, ::3] = float("nan")
    _check(x)


def test_misleading_sample_takes_the_lsd_path():
    # every strided sample position (i * n / 8192) holds 0.5: all splitters equal, so two buckets
    # of ~n / 2 distinct keys each exceed the LDS capacity
    n = 1 << 20
    g = torch.Generator().manual_seed(9)
    x = torch.rand(1, n, generator=g)
    pos = (torch.arange(8192) * n) // 8192
    x[0, pos] = 0.5
    _check(x)
    t = torch.randint(0, 2, (n,), generator=g)
    _check(x, t, 1)


def test_binary_auroc_matches_cpu_on_bucket_path():
    from torcheval_amd.metrics.functional import binary_auprc, binary_auroc

    g = torch.Generator().manual_seed(11)
    for kind in ("uniform", "ties40", "sigmoid_confident"):
        x = _gen(kind, 1_000_000, 21)[0]
        t = torch.randint(0, 2, x.shape, generator=g)
        for fn in (binary_auroc, binary_auprc):
            got = float(fn(x.to(DEV), t.to(DEV)))
            want = float(fn(x.double(), t))
            assert got == pytest.approx(want, abs=1e-6), (kind, fn.__name__)
