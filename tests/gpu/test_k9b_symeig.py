"""K9b symmetric eigenvalues (on-chip Householder reduction + multisection) vs CPU fp64
``torch.linalg.eigvalsh``, and the FID compute built on it."""

import pytest
import torch

from torcheval_amd.metrics.image.fid import _tr_sqrt_product, frechet_distance, sym_eigvalsh
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _native_eig(m: torch.Tensor) -> torch.Tensor:
    lam = torch.empty(m.shape[0], dtype=torch.float64, device=DEV)
    status = torch.zeros(1, dtype=torch.int32, device=DEV)
    rc = native().sym_eigvals(m.contiguous(), lam, status)
    assert rc == 0, "K9b did not launch"
    assert int(status.item()) == 0, "K9b grid aborted"
    return lam.cpu()


def _spd(n: int, seed: int, rank: int = None) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, rank or n + 7, generator=g, dtype=torch.float64)
    return x @ x.T / x.shape[1]


@pytest.mark.parametrize("n", [3, 4, 5, 17, 64, 255, 256, 257, 1000, 2048])
def test_random_spd(n):
    m = _spd(n, n)
    ref = torch.linalg.eigvalsh(m)
    got = _native_eig(m.to(DEV))
    scale = ref.abs().max()
    torch.testing.assert_close(got, ref, rtol=0, atol=float(1e-12 * n * scale))


@pytest.mark.parametrize("n", [6, 300, 2048])
def test_indefinite_and_clustered(n):
    g = torch.Generator().manual_seed(7)
    q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    lam = torch.cat([torch.full((n // 3,), 2.0), torch.linspace(-5, 5, n - n // 3, dtype=torch.float64)])
    m = (q * lam) @ q.T
    m = (m + m.T) / 2
    ref = torch.linalg.eigvalsh(m)
    got = _native_eig(m.to(DEV))
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-12 * n * 5)


@pytest.mark.parametrize("n", [129, 384])  # 384: the grid hands its last 128 columns to the one-workgroup tail
@pytest.mark.parametrize("kind", ["zeros", "identity", "diagonal", "rank3", "tridiagonal"])
def test_structured(kind, n):
    if kind == "zeros":
        m = torch.zeros(n, n, dtype=torch.float64)
    elif kind == "identity":
        m = torch.eye(n, dtype=torch.float64) * 3.0
    elif kind == "diagonal":
        m = torch.diag(torch.arange(n, dtype=torch.float64) - 40.0)
    elif kind == "rank3":
        m = _spd(n, 3, rank=3)
    else:
        m = torch.diag(torch.full((n,), 2.0, dtype=torch.float64))
        m += torch.diag(torch.full((n - 1,), -1.0, dtype=torch.float64), 1)
        m += torch.diag(torch.full((n - 1,), -1.0, dtype=torch.float64), -1)
    ref = torch.linalg.eigvalsh(m)
    got = _native_eig(m.to(DEV))
    scale = max(float(ref.abs().max()), 1.0)
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-12 * n * scale)


@pytest.mark.parametrize("n", [256, 257, 383, 640])
def test_tail_block_boundaries(n):
    # the grid reduction stops at column n - 128 and the tail kernel finishes the trailing block:
    # spectra whose trailing block is already diagonal (zero reflectors in the tail), or couples
    # to the leading block only through one entry
    m = _spd(n, n)
    m[n - 128 :, n - 128 :] = torch.diag(torch.linspace(-3, 3, 128, dtype=torch.float64))
    m[n - 128 :, : n - 128] = 0.0
    m[: n - 128, n - 128 :] = 0.0
    m[n - 1, 0] = m[0, n - 1] = 0.5
    for mat in (m, _spd(n, n + 1)):
        ref = torch.linalg.eigvalsh(mat)
        got = _native_eig(mat.to(DEV))
        torch.testing.assert_close(got, ref, rtol=0, atol=1e-12 * n * max(float(ref.abs().max()), 1.0))


def test_repeated_calls_reuse_workspace():
    a, b = _spd(512, 1), _spd(300, 2)
    for _ in range(3):
        torch.testing.assert_close(_native_eig(a.to(DEV)), torch.linalg.eigvalsh(a), rtol=0, atol=1e-9)
        torch.testing.assert_close(_native_eig(b.to(DEV)), torch.linalg.eigvalsh(b), rtol=0, atol=1e-9)


def test_fid_trace_sqrt_matches_cpu():
    # FID-shaped covariances (D = 2048 from 3000 samples), tr sqrt(S1 S2) vs the CPU path
    d = 2048
    g = torch.Generator().manual_seed(0)
    x1 = torch.randn(3000, d, generator=g, dtype=torch.float64)
    x2 = torch.randn(3000, d, generator=g, dtype=torch.float64) * 1.3 + 0.1
    s1, s2 = torch.cov(x1.T), torch.cov(x2.T)
    ref = _tr_sqrt_product(s1, s2)
    got = _tr_sqrt_product(s1.to(DEV), s2.to(DEV)).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-10, atol=0)
    mu1, mu2 = x1.mean(0), x2.mean(0)
    torch.testing.assert_close(
        frechet_distance(mu1.to(DEV), s1.to(DEV), mu2.to(DEV), s2.to(DEV)).cpu(),
        frechet_distance(mu1, s1, mu2, s2),
        rtol=1e-9,
        atol=1e-9,
    )


def test_fallback_sizes():
    # sizes K9b does not take still go through sym_eigvalsh (rocSOLVER)
    for n in (1, 2, 2600):
        m = _spd(n, 5).to(DEV)
        torch.testing.assert_close(sym_eigvalsh(m).cpu(), torch.linalg.eigvalsh(m.cpu()), rtol=0, atol=1e-9)


# ----------------------------------------------------------------------------- K9c
@pytest.mark.parametrize("n", [2, 3, 63, 64, 65, 200, 1000, 2048])
def test_blocked_cholesky_matches_cpu(n):
    from torcheval_amd.metrics.image.fid import cholesky_ex

    m = _spd(n, 100 + n)
    L, info = cholesky_ex(m.to(DEV))
    assert int(info) == 0
    ref = torch.linalg.cholesky(m)
    torch.testing.assert_close(L.cpu(), ref, rtol=1e-10, atol=1e-10 * float(ref.abs().max()))
    assert torch.equal(L.cpu().triu(1), torch.zeros(n, n, dtype=torch.float64))


@pytest.mark.parametrize("n,bad", [(50, 10), (300, 0), (300, 150), (2048, 2000)])
def test_blocked_cholesky_reports_non_pd(n, bad):
    from torcheval_amd.metrics.image.fid import cholesky_ex

    m = _spd(n, 7)
    m[bad, bad] = -1.0  # a leading minor of order bad + 1 is indefinite
    _, info = cholesky_ex(m.to(DEV))
    _, ref_info = torch.linalg.cholesky_ex(m)
    assert int(info) != 0 and int(ref_info) != 0
    assert int(info) <= bad + 1


@pytest.mark.parametrize("n", [2049, 2304, 2560])
def test_largest_instances(n):
    # the 9 x 9 and 10 x 10 register instances (n > 2048): more rows and columns per thread
    m = _spd(n, n)
    ref = torch.linalg.eigvalsh(m)
    got = _native_eig(m.to(DEV))
    torch.testing.assert_close(got, ref, rtol=0, atol=float(1e-12 * n * ref.abs().max()))


@pytest.mark.parametrize("payload", ["default", "all_ones"])
def test_nan_entries_do_not_stall_the_hand_off(payload):
    # a NaN is canonicalised before it is handed off, so no stored value can equal the
    # all-one-bytes sentinel of an unpublished slot - not even a NaN input that carries
    # exactly that bit pattern; the launch completes (status 0) and the eigenvalues are NaN
    m = _spd(300, 3)
    bad = torch.tensor([-1], dtype=torch.int64).view(torch.float64)[0] if payload == "all_ones" else float("nan")
    m[10, 20] = m[20, 10] = bad
    lam = torch.empty(300, dtype=torch.float64, device=DEV)
    status = torch.zeros(1, dtype=torch.int32, device=DEV)
    assert native().sym_eigvals(m.to(DEV), lam, status) == 0
    assert int(status.item()) == 0
    assert torch.isnan(lam.cpu()).all()


_WAVE_CHILD = r"""
import torch
from torcheval_amd.ops import native
out = []
for n in (3, 5, 64, 257, 1000, 2048):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, n + 7, generator=g, dtype=torch.float64)
    m = x @ x.T / x.shape[1]
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert native().sym_eigvals(m.cuda(), lam, st) == 0 and int(st.item()) == 0
    ref = torch.linalg.eigvalsh(m)
    out.append(float((lam.cpu() - ref).abs().max() / ref.abs().max()))
print(max(out))
"""


def test_wave_kernel_arm_matches_cpu():
    """The opt-in rows-per-wave reduction (TORCHEVAL_AMD_SYMEIG_WAVE=1, read once per process,
    hence the child process) against CPU eigvalsh."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, TORCHEVAL_AMD_SYMEIG_WAVE="1")
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", _WAVE_CHILD], env=env, cwd=root, capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert float(r.stdout.strip().splitlines()[-1]) < 1e-12
