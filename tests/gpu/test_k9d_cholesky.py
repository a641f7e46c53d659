"""K9d one-launch blocked Cholesky (csrc/kernels/cholesky.hip), the triangle-aware L^T S L and
the FP64 covariance pass (csrc/kernels/fid_prep.hip) against CPU fp64 references; FID compute
end to end against the ATen formulation (reference torcheval/metrics/image/fid.py:192-262)."""

import pytest
import torch

from torcheval_amd.metrics.image.fid import (
    FrechetInceptionDistance,
    _chol,
    _covariance,
    _lt_s_l,
    frechet_distance,
)
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _spd(n: int, seed: int, rank: int = None) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, rank or n + 7, generator=g, dtype=torch.float64)
    return x @ x.T / x.shape[1]


@pytest.mark.parametrize("n", [1, 5, 64, 127, 128, 129, 700, 2048, 2500])
def test_factor_matches_cpu(n):
    m = _spd(n, 300 + n)
    L, info = _chol(m.to(DEV))
    assert info == 0
    ref = torch.linalg.cholesky(m)
    Lc = L.cpu()
    torch.testing.assert_close(Lc, ref, rtol=1e-10, atol=1e-11 * float(ref.abs().max()))
    assert torch.equal(Lc.triu(1), torch.zeros(n, n, dtype=torch.float64))


def test_padding_and_views():
    # a strided (non-contiguous-row-stride) input and a repeated call reuse nothing stale
    big = _spd(300, 9)
    m = big[:250, :250]  # row stride 300
    for _ in range(3):
        L, info = _chol(m.to(DEV)[:, :])
        assert info == 0
        torch.testing.assert_close(L.cpu(), torch.linalg.cholesky(m), rtol=1e-10, atol=1e-12)
    mv = big.to(DEV)[:250, :250]
    L, info = _chol(mv)
    assert info == 0
    torch.testing.assert_close(L.cpu(), torch.linalg.cholesky(m), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("n,bad", [(64, 0), (64, 63), (200, 130), (2048, 1500), (2048, 64)])
def test_non_pd_reports_first_column(n, bad):
    m = _spd(n, 5)
    m[bad, bad] = -1.0
    _, info = _chol(m.to(DEV))
    _, ref_info = torch.linalg.cholesky_ex(m)
    assert info != 0 and int(ref_info) != 0
    assert info <= bad + 1


def test_nan_input_completes():
    # NaNs are canonicalised before publication, so no hand-off waits forever on a sentinel
    m = _spd(300, 4)
    m[10, 20] = m[20, 10] = float("nan")
    m[200, 5] = m[5, 200] = torch.tensor([-1], dtype=torch.int64).view(torch.float64)[0]  # all-one bits
    a = m.to(DEV)
    nt = native().cholesky_tiles(300)
    L = torch.empty(64 * nt, 64 * nt, dtype=torch.float64, device=DEV)
    linv = torch.empty(nt * 4096, dtype=torch.float64, device=DEV)
    ctl = torch.empty(1, dtype=torch.int32, device=DEV)
    st = torch.empty(2, dtype=torch.int32, device=DEV)
    native().cholesky_factor(a, L, linv, ctl, st)
    assert int(st[1].item()) == 0  # no abort


@pytest.mark.parametrize("n", [100, 512, 1000, 2048])
def test_triangle_aware_sandwich(n):
    L = torch.linalg.cholesky(_spd(n, 11))
    s = _spd(n, 12)
    ref = L.T @ s @ L
    got = _lt_s_l(L.to(DEV), s.to(DEV))
    g = got.cpu()
    assert torch.equal(g, g.T)  # exactly symmetric
    torch.testing.assert_close(g, ref, rtol=1e-11, atol=1e-12 * float(ref.abs().max()))


@pytest.mark.parametrize("d,n", [(17, 40), (64, 500), (2048, 3000), (1000, 999)])
def test_covariance_pass(d, n):
    g = torch.Generator().manual_seed(d)
    x = torch.randn(n, d, generator=g) * 2 + 0.5
    cov_sum = (x.T @ x).float()
    cov_sum[3 % d, 7 % d] += 0.25  # a non-symmetric state is symmetrised
    col = x.sum(0).float()
    got = _covariance(cov_sum.to(DEV), col.to(DEV), n).cpu()
    assert torch.equal(got, got.T)
    mean = col.double() / n
    ref = (cov_sum.double() - n * torch.outer(mean, mean)) / (n - 1)
    ref = (ref + ref.T) / 2
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12 * float(ref.abs().max()))


def test_fid_compute_end_to_end():
    d = 2048
    fid = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=d, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(3)
    for real, scale in ((True, 1.0), (False, 1.1)):
        for _ in range(2):
            fid.update_activations(torch.randn(4096, d, device=DEV, generator=g) * scale + 0.05, real)
    got = float(fid.compute())
    nr, nf = int(fid.num_real_images), int(fid.num_fake_images)
    rm, fm = fid.real_sum.double().cpu() / nr, fid.fake_sum.double().cpu() / nf
    rc = (fid.real_cov_sum.double().cpu() - nr * torch.outer(rm, rm)) / (nr - 1)
    fc = (fid.fake_cov_sum.double().cpu() - nf * torch.outer(fm, fm)) / (nf - 1)
    want = float(frechet_distance(rm, rc, fm, fc))
    assert got == pytest.approx(want, rel=1e-6)
