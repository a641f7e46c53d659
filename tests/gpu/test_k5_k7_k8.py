"""K5 (column moments: MSE / R2), K7 (fused log-softmax perplexity), K8 (FP32-MFMA FID
covariance) and the families built on them, vs CPU fp64 references."""

import math

import pytest
import torch

from torcheval_amd.metrics import (
    FrechetInceptionDistance,
    MeanSquaredError,
    Perplexity,
    R2Score,
    WindowedBinaryNormalizedEntropy,
    WindowedMeanSquaredError,
)
from torcheval_amd.metrics.functional import (
    binary_normalized_entropy,
    mean_squared_error,
    perplexity,
    r2_score,
)
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


# ----------------------------------------------------------------------------- K5
@pytest.mark.parametrize("shape", [(1,), (1000,), (4097, 3), (100_003, 16), (64, 257)])
@pytest.mark.parametrize("weighted", [False, True])
def test_k5_mse_matches_cpu(shape, weighted):
    g = torch.Generator().manual_seed(sum(shape))
    x, y = torch.randn(shape, generator=g), torch.randn(shape, generator=g)
    w = torch.rand(shape[0], generator=g) if weighted else None
    for mo in ("uniform_average", "raw_values"):
        ref = mean_squared_error(x.double(), y.double(), sample_weight=None if w is None else w.double(), multioutput=mo)
        got = mean_squared_error(x.to(DEV), y.to(DEV), sample_weight=None if w is None else w.to(DEV), multioutput=mo)
        torch.testing.assert_close(got.cpu().double(), ref, rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.int64])
def test_k5_mixed_dtypes(dtype):
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(5000, 4, generator=g) * 3).to(dtype)
    y = torch.randn(5000, 4, generator=g)
    ref = mean_squared_error(x.double(), y.double())
    got = mean_squared_error(x.to(DEV), y.to(DEV))
    torch.testing.assert_close(got.cpu().double(), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mo", ["uniform_average", "raw_values", "variance_weighted"])
def test_k5_r2_matches_cpu(mo):
    g = torch.Generator().manual_seed(11)
    x, y = torch.randn(20000, 5, generator=g), torch.randn(20000, 5, generator=g) + 2
    ref = r2_score(x.double(), y.double(), multioutput=mo)
    got = r2_score(x.to(DEV), y.to(DEV), multioutput=mo)
    torch.testing.assert_close(got.cpu().double(), ref, rtol=1e-4, atol=1e-5)
    m = R2Score(multioutput=mo, device=DEV)
    for i in range(4):
        m.update(x[i::4].to(DEV), y[i::4].to(DEV))
    torch.testing.assert_close(m.compute().cpu().double(), ref, rtol=1e-4, atol=1e-5)


def test_k5_class_and_window():
    g = torch.Generator().manual_seed(12)
    xs = [torch.randn(3000, generator=g) for _ in range(6)]
    ys = [torch.randn(3000, generator=g) for _ in range(6)]
    m = MeanSquaredError(device=DEV)
    wm = WindowedMeanSquaredError(max_num_updates=2, device=DEV)
    for x, y in zip(xs, ys):
        m.update(x.to(DEV), y.to(DEV))
        wm.update(x.to(DEV), y.to(DEV))
    ref = mean_squared_error(torch.cat(xs).double(), torch.cat(ys).double())
    torch.testing.assert_close(m.compute().cpu().double(), ref, rtol=1e-5, atol=1e-6)
    life, win = wm.compute()
    torch.testing.assert_close(life.cpu().double(), ref, rtol=1e-5, atol=1e-6)
    ref_w = mean_squared_error(torch.cat(xs[-2:]).double(), torch.cat(ys[-2:]).double())
    torch.testing.assert_close(win.cpu().double(), ref_w, rtol=1e-5, atol=1e-6)


# ----------------------------------------------------------------------------- K7
def _ppl_ref(x, t, ignore=None):
    lp = torch.log_softmax(x.double().reshape(-1, x.shape[-1]), -1)
    tt = t.reshape(-1)
    keep = tt != ignore if ignore is not None else torch.ones_like(tt, dtype=torch.bool)
    return math.exp(-float(lp[keep].gather(1, tt[keep, None]).sum()) / int(keep.sum()))


@pytest.mark.parametrize("vocab", [3, 17, 1001, 32000, 50257])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_k7_perplexity_matches_fp64(vocab, dtype):
    g = torch.Generator().manual_seed(vocab)
    x = (torch.randn(4, 33, vocab, generator=g) * 4).to(dtype)
    t = torch.randint(0, vocab, (4, 33), generator=g)
    ref = _ppl_ref(x, t)
    got = float(perplexity(x.to(DEV), t.to(DEV)))
    assert got == pytest.approx(ref, rel=2e-5)
    ign = int(t[0, 0])
    assert float(perplexity(x.to(DEV), t.to(DEV), ignore_index=ign)) == pytest.approx(_ppl_ref(x, t, ign), rel=2e-5)


def test_k7_strided_rows_and_class():
    g = torch.Generator().manual_seed(5)
    big = torch.randn(2, 16, 1024 + 64, generator=g)
    x = big[..., :1024]  # row stride != vocab
    t = torch.randint(0, 1024, (2, 16), generator=g)
    assert float(perplexity(x.to(DEV), t.to(DEV))) == pytest.approx(_ppl_ref(x, t), rel=2e-5)
    m = Perplexity(device=DEV)
    m.update(x.to(DEV), t.to(DEV))
    m.update(x.to(DEV) * 0.5, t.to(DEV))
    ref = _ppl_ref(torch.cat([x, x * 0.5]), torch.cat([t, t]))
    assert float(m.compute()) == pytest.approx(ref, rel=2e-5)


@pytest.mark.parametrize("vocab", [4096, 4112, 8192, 12288, 12304])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_k7_long_row_chunk_edges(vocab, dtype):
    """Long rows stream in 1024-value wave-wide chunks: rows of exactly 4, 8 and 12 chunks and of
    4 and 12 chunks plus a 16-value tail, with the max in the last chunk of one row."""
    g = torch.Generator().manual_seed(vocab + 7)
    x = (torch.randn(3, 11, vocab, generator=g) * 4).to(dtype)
    x[0, 0, vocab - 1] = 40.0  # the max sits in the last chunk of one row
    t = torch.randint(0, vocab, (3, 11), generator=g)
    t[0, 0] = vocab - 1
    got = float(perplexity(x.to(DEV), t.to(DEV)))
    assert got == pytest.approx(_ppl_ref(x, t), rel=2e-5)
    ign = int(t[1, 3])
    got_i = float(perplexity(x.to(DEV), t.to(DEV), ignore_index=ign))
    assert got_i == pytest.approx(_ppl_ref(x, t, ign), rel=2e-5)


def test_k7_many_long_rows_strided_and_deterministic():
    from torcheval_amd.config import flags

    g = torch.Generator().manual_seed(11)
    big = torch.randn(2, 4100, 4096 + 32, generator=g)  # grid-stride: more rows than waves in the grid
    x = big[..., :4096]  # row stride != vocab
    t = torch.randint(0, 4096, (2, 4100), generator=g)
    ref = _ppl_ref(x, t)
    xd, td = x.to(DEV), t.to(DEV)
    got = float(perplexity(xd, td))
    assert got == pytest.approx(ref, rel=2e-5)
    with flags(deterministic=True):
        a = perplexity(xd, td)
        b = perplexity(xd, td)
    assert float(a) == pytest.approx(ref, rel=2e-5)
    assert torch.equal(a, b)


@pytest.mark.parametrize("off", [1, 2, 3, 5])
@pytest.mark.parametrize("vocab", [3, 5, 40, 1000, 50257])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_k7_split_rows_head_body_tail(off, vocab, dtype):
    """Rows that do not start 16-B aligned (column offset into a wider buffer, odd vocab) take
    the scalar head / 16-B body / scalar tail split; the max sits in the head of one row and
    in the tail of another, and V smaller than the head is covered by vocab 3 and 5."""
    g = torch.Generator().manual_seed(off * 100 + vocab)
    big = (torch.randn(3, 37, vocab + off + 7, generator=g) * 4).to(dtype)
    x = big[..., off:off + vocab]
    x[0, 0, 0] = 40.0
    x[0, 1, vocab - 1] = 40.0
    t = torch.randint(0, vocab, (3, 37), generator=g)
    t[0, 0], t[0, 1] = 0, vocab - 1
    xd = big.to(DEV)[..., off:off + vocab]
    got = float(perplexity(xd, t.to(DEV)))
    assert got == pytest.approx(_ppl_ref(x, t), rel=2e-5)


def test_k7_long_row_invalid_target_raises():
    x = torch.randn(2, 2, 4096, device=DEV)
    with pytest.raises(ValueError, match="vocab_size minus one"):
        perplexity(x, torch.tensor([[1, 4096], [0, 3]], device=DEV))


def test_k7_invalid_target_raises():
    with pytest.raises(ValueError, match="vocab_size minus one"):
        perplexity(torch.rand(3, 2, 3, device=DEV), torch.tensor([[4, 2], [1, 0], [0, 0]], device=DEV))


# ----------------------------------------------------------------------------- K8
@pytest.mark.parametrize("n,d", [(1, 8), (37, 100), (64, 128), (200, 300), (256, 2048), (1000, 2048), (50, 37), (300, 1001)])
def test_k8_cov_matches_fp64(n, d):
    g = torch.Generator().manual_seed(n * 7 + d)
    act = torch.randn(n, d, generator=g)
    cov0 = torch.randn(d, d, generator=g)
    cov0 = cov0 + cov0.T
    s0 = torch.randn(d, generator=g)
    cov, s = cov0.to(DEV), s0.to(DEV)
    native().fid_cov_update(act.to(DEV), cov, s)
    torch.cuda.synchronize()
    ref = cov0.double() + act.double().T @ act.double()
    torch.testing.assert_close(cov.cpu().double(), ref, rtol=1e-4, atol=1e-3 * math.sqrt(n))
    torch.testing.assert_close(s.cpu().double(), s0.double() + act.double().sum(0), rtol=1e-5, atol=1e-3)
    # result must be exactly symmetric (mirrored tiles)
    c = cov.cpu() - cov0
    assert torch.equal(c, c.T)


@pytest.mark.parametrize("n,d,split", [(5000, 512, 0), (1000, 2048, 3), (333, 300, 2), (70, 2048, 5)])
def test_k8_split_k_matches_fp64(n, d, split, monkeypatch):
    """split-K items (partials + fix-up pass): auto split for a small D, forced splits
    (including one with an empty last K-range) for the others."""
    if split:
        monkeypatch.setenv("TORCHEVAL_AMD_K8_SPLIT", str(split))
    g = torch.Generator().manual_seed(n + d)
    act = torch.randn(n, d, generator=g)
    cov0 = torch.randn(d, d, generator=g)
    cov0 = cov0 + cov0.T
    s0 = torch.randn(d, generator=g)
    cov, s = cov0.to(DEV), s0.to(DEV)
    native().fid_cov_update(act.to(DEV), cov, s)
    torch.cuda.synchronize()
    ref = cov0.double() + act.double().T @ act.double()
    torch.testing.assert_close(cov.cpu().double(), ref, rtol=1e-4, atol=1e-3 * math.sqrt(n))
    torch.testing.assert_close(s.cpu().double(), s0.double() + act.double().sum(0), rtol=1e-5, atol=1e-3)
    c = cov.cpu() - cov0
    assert torch.equal(c, c.T)
    again = cov0.to(DEV)
    native().fid_cov_update(act.to(DEV), again, None)
    assert torch.equal(again.cpu(), cov.cpu())  # deterministic for a given split


K8_MODES = ("shared", "wave", "exact")  # kMode 2 (default), 1, 0 of fid_cov.hip


def _k8_mode(monkeypatch, mode: str) -> None:
    monkeypatch.delenv("TORCHEVAL_AMD_K8_EXACT", raising=False)
    monkeypatch.delenv("TORCHEVAL_AMD_K8_MODE", raising=False)
    if mode == "exact":
        monkeypatch.setenv("TORCHEVAL_AMD_K8_EXACT", "1")
    elif mode == "wave":
        monkeypatch.setenv("TORCHEVAL_AMD_K8_MODE", "1")


@pytest.mark.parametrize("n,d", [(1000, 2048), (333, 300), (64, 128), (130, 2048)])
def test_k8_split_bf16_exact_on_integers(n, d, monkeypatch):
    """Small-integer activations: every product and partial sum is exact in FP32, so the bf16
    three-way-split path must reproduce the integer result bit for bit (catches any fragment
    k-order / lane-map mistake), in both MFMA modes."""
    g = torch.Generator().manual_seed(n + 3 * d)
    act = torch.randint(-8, 9, (n, d), generator=g).float()
    want = (act.long().T @ act.long()).float()
    for mode in K8_MODES:
        _k8_mode(monkeypatch, mode)
        cov = torch.zeros(d, d, device=DEV)
        s = torch.zeros(d, device=DEV)
        native().fid_cov_update(act.to(DEV), cov, s)
        assert torch.equal(cov.cpu(), want), mode
        assert torch.equal(s.cpu(), act.sum(0)), mode


@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e4])
def test_k8_split_bf16_error_matches_fp32_mfma(scale, monkeypatch):
    """The bf16 split path's error against fp64 stays at the FP32-MFMA path's level (the
    dropped split products are below 2^-23 |xy|), over a wide dynamic range of activations."""
    g = torch.Generator().manual_seed(11)
    act = (torch.randn(1000, 2048, generator=g) * torch.exp(torch.randn(1, 2048, generator=g) * 2)) * scale
    ref = act.double().T @ act.double()
    errs = {}
    bound = act.double().abs().T @ act.double().abs()
    for mode in K8_MODES:
        _k8_mode(monkeypatch, mode)
        cov = torch.zeros(2048, 2048, device=DEV)
        native().fid_cov_update(act.to(DEV), cov, None)
        d = (cov.cpu().double() - ref).abs()
        # per-element error relative to sum_k |x_ik x_jk|, the scale of FP32 rounding
        errs[mode] = float((d / bound).max())
    for mode in ("shared", "wave"):
        assert errs[mode] < 2 * errs["exact"] + 1e-7, errs
        assert errs[mode] < 2e-6, errs


def test_k8_strided_activations():
    g = torch.Generator().manual_seed(3)
    big = torch.randn(50, 2048 + 32, generator=g)
    act = big[:, :2048]
    cov = torch.zeros(2048, 2048, device=DEV)
    native().fid_cov_update(act.to(DEV), cov, None)
    torch.testing.assert_close(cov.cpu().double(), act.double().T @ act.double(), rtol=1e-4, atol=1e-2)


def test_fid_class_gpu_matches_cpu():
    torch.manual_seed(0)
    d = 256

    class Feat(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.register_buffer("p", torch.randn(3 * 64, d))

        def forward(self, x):
            return torch.nn.functional.adaptive_avg_pool2d(x, 8).flatten(1) @ self.p

    model = Feat()
    real, fake = torch.rand(96, 3, 16, 16), torch.rand(96, 3, 16, 16) ** 2
    cpu = FrechetInceptionDistance(model=model, feature_dim=d)
    gpu = FrechetInceptionDistance(model=Feat().to(DEV), feature_dim=d, device=DEV)
    gpu.model.load_state_dict(model.state_dict())
    for i in range(3):
        sl = slice(32 * i, 32 * (i + 1))
        cpu.update(real[sl], True).update(fake[sl], False)
        gpu.update(real[sl].to(DEV), True).update(fake[sl].to(DEV), False)
    torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-3, atol=1e-2)


def test_fid_default_inception_gpu():
    with pytest.warns(RuntimeWarning):
        m = FrechetInceptionDistance(device=DEV)
    imgs = torch.rand(4, 3, 299, 299, device=DEV)
    m.update(imgs, True).update(imgs.flip(-1), False)
    v = m.compute()
    assert torch.isfinite(v)


# ----------------------------------------------------------------------------- window on GPU (K6)
def test_windowed_ne_gpu():
    g = torch.Generator().manual_seed(9)
    m = WindowedBinaryNormalizedEntropy(num_tasks=2, max_num_updates=3, device=DEV)
    xs, ts = [], []
    for _ in range(5):
        x, t = torch.rand(2, 500, generator=g), torch.randint(0, 2, (2, 500), generator=g).float()
        m.update(x.to(DEV), t.to(DEV))
        xs.append(x), ts.append(t)
    life, win = m.compute()
    torch.testing.assert_close(life.cpu(), binary_normalized_entropy(torch.cat(xs, 1).double(), torch.cat(ts, 1).double(), num_tasks=2), rtol=1e-6, atol=1e-8)
    torch.testing.assert_close(win.cpu(), binary_normalized_entropy(torch.cat(xs[-3:], 1).double(), torch.cat(ts[-3:], 1).double(), num_tasks=2), rtol=1e-6, atol=1e-8)


def test_k8_misaligned_contiguous_view():
    """A contiguous activation view at a 4-byte storage offset is re-allocated (16-B aligned)
    before K8, instead of tripping the kernel's alignment check."""
    from torcheval_amd.metrics.image.fid import FrechetInceptionDistance

    base = torch.rand(257 * 64 + 1, device=DEV)
    act = base[1:].view(257, 64)
    assert act.is_contiguous() and act.data_ptr() % 16 != 0
    m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=64, device=DEV)
    m.update_activations(act, True)
    ref = act.double().T @ act.double()
    torch.testing.assert_close(m.real_cov_sum.double(), ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(m.real_sum.double(), act.double().sum(0), rtol=1e-5, atol=1e-4)


def test_fid_staged_updates_match_direct(monkeypatch):
    """Staged FID updates (one copy per update, K8 once per 8192-row stage or on read) give
    the states of per-update K8 launches; the 10 real x 1000-row stream crosses one full stage."""
    from torcheval_amd.metrics.image import fid as fid_mod

    g = torch.Generator(device=DEV).manual_seed(5)
    acts = [torch.rand(1000, 2048, device=DEV, generator=g) for _ in range(12)]
    staged = fid_mod.FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=DEV)
    for i, a in enumerate(acts):
        staged.update_activations(a, i % 6 != 5)
    assert staged._stage_rows == [2000, 2000]  # real flushed once at 8000 rows; the rest pending
    monkeypatch.setattr(fid_mod, "_stageable", lambda act: False)
    direct = fid_mod.FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=DEV)
    for i, a in enumerate(acts):
        direct.update_activations(a, i % 6 != 5)
    assert direct._stage_rows == [0, 0]
    for name in ("real_sum", "real_cov_sum", "fake_sum", "fake_cov_sum"):
        torch.testing.assert_close(getattr(staged, name), getattr(direct, name), rtol=1e-4, atol=1e-2)
    assert int(staged.num_real_images) == 10000 and int(staged.num_fake_images) == 2000
    real = torch.cat([a for i, a in enumerate(acts) if i % 6 != 5]).double()
    torch.testing.assert_close(staged.real_cov_sum.double(), real.T @ real, rtol=1e-4, atol=1e-1)
    torch.testing.assert_close(staged.compute(), direct.compute(), rtol=1e-3, atol=1e-4)
