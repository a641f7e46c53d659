"""K9p pivoted (rank-revealing) FP64 Cholesky (csrc/kernels/pivchol.hip) and the rank-deficient
FID compute built on it, against FP64 CPU references: the eigh factorisation the path replaced
(``_eigh_factor``) and LAPACK-semantics properties of the factor (reference
torcheval/metrics/image/fid.py:192-230 takes any rank through ``linalg.eigvals``)."""

import pytest
import torch

from torcheval_amd.metrics.image.fid import (
    FrechetInceptionDistance,
    _eigh_factor,
    _pivoted_factor,
    _tr_sqrt_product,
)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _low_rank(n: int, r: int, seed: int, scale: float = 1.0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(r, n, generator=g, dtype=torch.float64) * scale
    s = x.T @ x / max(r, 1)
    return (s + s.T) / 2


def _cov(samples: int, d: int, seed: int, scale: float = 1.0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(samples, d, generator=g, dtype=torch.float64) * scale + 0.1
    c = torch.cov(x.T)
    return (c + c.T) / 2


def _tr_sqrt_eigh(s1: torch.Tensor, s2: torch.Tensor) -> float:
    w = _eigh_factor(s1)
    m = w @ s2 @ w.T
    return float(torch.linalg.eigvalsh((m + m.T) / 2).clamp(min=0).sqrt().sum())


@pytest.mark.parametrize("n,r", [(1, 1), (5, 2), (64, 10), (100, 99), (700, 300), (1024, 500), (1025, 1025),
                                 (1500, 1000), (2048, 999)])
def test_factor_reconstructs_and_reveals_rank(n, r):
    s = _low_rank(n, r, 10 + n)
    w = _pivoted_factor(s.to(DEV))
    assert w is not None
    wc = w.cpu()
    assert wc.shape == (r, n)
    scale = float(s.diagonal().max())
    torch.testing.assert_close(wc.T @ wc, s, rtol=0, atol=1e-12 * scale)


def test_zero_and_identity():
    z = _pivoted_factor(torch.zeros(70, 70, dtype=torch.float64, device=DEV))
    assert z.shape == (0, 70)
    e = _pivoted_factor(torch.eye(130, dtype=torch.float64, device=DEV) * 3.0).cpu()
    assert e.shape == (130, 130)
    torch.testing.assert_close(e.T @ e, torch.eye(130, dtype=torch.float64) * 3.0, rtol=0, atol=1e-14)


def test_nan_gives_nan():
    s = _low_rank(200, 50, 3)
    s[7, 9] = s[9, 7] = float("nan")
    w = _pivoted_factor(s.to(DEV))
    assert w is not None and bool(torch.isnan(w).any())


def test_deterministic():
    s = _cov(500, 1200, 4).to(DEV)
    a, b = _pivoted_factor(s), _pivoted_factor(s)
    assert torch.equal(a, b)


# r1 <= r2 and both < d: W S2 W^T (r1 x r1) is then generically of full rank, so its square-rooted
# spectrum has no rounding-level eigenvalues (whose square roots no method pins below ~1e-8)
@pytest.mark.parametrize("d,r1,r2", [(512, 200, 300), (2048, 999, 999), (1000, 400, 600)])
def test_tr_sqrt_matches_eigh_constructed_rank(d, r1, r2):
    s1, s2 = _low_rank(d, r1, 20 + d), _low_rank(d, r2, 30 + d, 1.3)
    got = float(_tr_sqrt_product(s1.to(DEV), s2.to(DEV)))
    want = _tr_sqrt_eigh(s1, s2)
    assert got == pytest.approx(want, rel=1e-10)


def test_tr_sqrt_matches_eigh_standin_activations():
    # the suite's shape: 1000 + 1000 activation rows at D = 2048, FP64 covariances
    s1, s2 = _cov(1000, 2048, 41), _cov(1000, 2048, 42, 1.1)
    got = float(_tr_sqrt_product(s1.to(DEV), s2.to(DEV), 1000, 1000))
    want = _tr_sqrt_eigh(s1, s2)
    assert got == pytest.approx(want, rel=1e-10)


def test_fid_class_singular_end_to_end():
    # FP32 states: the covariances carry FP32 rounding spectrum above the FP64 tolerance (kept by
    # both factorisations, as the reference's eigvals keeps it); both sit within the FP32
    # state noise of the FP64 truth (scipy-style oracle on the exact covariances)
    d, n = 2048, 1000
    g = torch.Generator().manual_seed(7)
    real = torch.randn(n, d, generator=g)
    fake = torch.randn(n, d, generator=g) * 1.1 + 0.05
    m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=d, device=DEV)
    m.update_activations(real.to(DEV), True).update_activations(fake.to(DEV), False)
    got = float(m.compute())
    r, f = real.double(), fake.double()
    s1, s2 = torch.cov(r.T), torch.cov(f.T)
    want = float((r.mean(0) - f.mean(0)).square().sum() + s1.trace() + s2.trace() - 2 * _tr_sqrt_eigh(s1, s2))
    assert got == pytest.approx(want, rel=2e-3)


def test_one_side_singular_uses_cholesky_of_other():
    # L2^T S1 L2 is D x D of rank 100: its 200 rounding-level eigenvalues put ~1e-8 into the sum
    d = 300
    s1, s2 = _low_rank(d, 100, 51), _cov(2000, d, 52)
    got = float(_tr_sqrt_product(s1.to(DEV), s2.to(DEV), 101, 2000))
    assert got == pytest.approx(_tr_sqrt_eigh(s1, s2), rel=1e-6)


def test_unsupported_size_falls_back():
    s = _low_rank(2100, 50, 61)
    assert _pivoted_factor(s.to(DEV)) is None
    got = float(_tr_sqrt_product(s.to(DEV), _low_rank(2100, 60, 62).to(DEV)))
    assert got == pytest.approx(_tr_sqrt_eigh(s, _low_rank(2100, 60, 62)), rel=1e-9)
