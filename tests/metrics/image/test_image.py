"""PSNR and FID (parity: tests/metrics/image/test_psnr.py, test_fid.py).

FID is checked against an independent scipy ``sqrtm`` implementation of the Frechet distance
(no pretrained Inception weights exist offline, so the feature extractor is a small fixed
module; the default model is exercised for shape/validation only)."""

import numpy as np
import pytest
import scipy.linalg
import torch
from torch import nn

from torcheval_amd.metrics import FrechetInceptionDistance, PeakSignalNoiseRatio
from torcheval_amd.metrics.functional import peak_signal_noise_ratio
from torcheval_amd.utils.test_utils import MetricClassTester


def _psnr_oracle(x: torch.Tensor, y: torch.Tensor, data_range=None) -> torch.Tensor:
    x, y = x.double().numpy(), y.double().numpy()
    rng = (y.max() - y.min()) if data_range is None else data_range
    mse = np.mean((x - y) ** 2)
    return torch.tensor(10 * np.log10(rng**2 / mse), dtype=torch.float32)


class TestPSNR(MetricClassTester):
    def test_functional(self) -> None:
        torch.manual_seed(0)
        x, y = torch.rand(4, 3, 16, 16), torch.rand(4, 3, 16, 16)
        torch.testing.assert_close(peak_signal_noise_ratio(x, y), _psnr_oracle(x, y), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(peak_signal_noise_ratio(x, y, 2.0), _psnr_oracle(x, y, 2.0), rtol=1e-5, atol=1e-5)

    def test_class_auto_range(self) -> None:
        torch.manual_seed(1)
        x, y = torch.rand(8, 4, 3, 8, 8), torch.rand(8, 4, 3, 8, 8) * 2 - 0.5
        self.run_class_implementation_tests(
            metric=PeakSignalNoiseRatio(),
            state_names={"data_range", "num_observations", "sum_squared_error", "min_target", "max_target"},
            update_kwargs={"input": x, "target": y},
            compute_result=_psnr_oracle(x, y),
            atol=1e-4,
        )

    def test_class_fixed_range(self) -> None:
        torch.manual_seed(2)
        x, y = torch.rand(8, 4, 3, 8, 8), torch.rand(8, 4, 3, 8, 8)
        self.run_class_implementation_tests(
            metric=PeakSignalNoiseRatio(data_range=1.0),
            state_names={"data_range", "num_observations", "sum_squared_error", "min_target", "max_target"},
            update_kwargs={"input": x, "target": y},
            compute_result=_psnr_oracle(x, y, 1.0),
            atol=1e-4,
        )

    def test_invalid(self) -> None:
        with pytest.raises(ValueError, match="`data_range needs to be either `None` or `float`."):
            PeakSignalNoiseRatio(data_range=1)
        with pytest.raises(ValueError, match="`data_range` needs to be positive."):
            peak_signal_noise_ratio(torch.rand(2), torch.rand(2), -1.0)
        with pytest.raises(ValueError, match="same shape"):
            peak_signal_noise_ratio(torch.rand(2, 3), torch.rand(3, 2))


class _Features(nn.Module):
    """Deterministic tiny feature extractor: 4x4 average pool + fixed projection."""

    def __init__(self, dim: int) -> None:
        super().__init__()
        g = torch.Generator().manual_seed(123)
        self.register_buffer("proj", torch.randn(3 * 16, dim, generator=g))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.nn.functional.adaptive_avg_pool2d(x, 4).flatten(1) @ self.proj


def _fid_oracle(real: np.ndarray, fake: np.ndarray) -> float:
    mu1, mu2 = real.mean(0), fake.mean(0)
    s1, s2 = np.cov(real, rowvar=False), np.cov(fake, rowvar=False)
    covmean = scipy.linalg.sqrtm(s1 @ s2)
    covmean = covmean.real
    return float(((mu1 - mu2) ** 2).sum() + np.trace(s1) + np.trace(s2) - 2 * np.trace(covmean))


class TestFID(MetricClassTester):
    def test_against_scipy(self) -> None:
        torch.manual_seed(3)
        d = 24
        model = _Features(d)
        real = torch.rand(8, 32, 3, 16, 16)
        fake = torch.rand(8, 32, 3, 16, 16) ** 2
        feats_r = torch.cat([model(b) for b in real]).double().numpy()
        feats_f = torch.cat([model(b) for b in fake]).double().numpy()
        expected = torch.tensor(_fid_oracle(feats_r, feats_f), dtype=torch.float32)
        m = FrechetInceptionDistance(model=model, feature_dim=d)
        for r, f in zip(real, fake):
            m.update(r, is_real=True).update(f, is_real=False)
        torch.testing.assert_close(m.compute(), expected, rtol=1e-3, atol=1e-3)

    def test_class_suite(self) -> None:
        torch.manual_seed(4)
        d = 12
        model = _Features(d)
        images = torch.rand(8, 16, 3, 8, 8)
        is_real = [True, False] * 4
        images[1::2] = images[1::2] ** 3
        feats = torch.stack([model(b) for b in images]).double()
        expected = _fid_oracle(
            feats[0::2].reshape(-1, d).numpy(), feats[1::2].reshape(-1, d).numpy()
        )
        self.run_class_implementation_tests(
            metric=FrechetInceptionDistance(model=model, feature_dim=d),
            state_names={"real_sum", "real_cov_sum", "fake_sum", "fake_cov_sum",
                         "num_real_images", "num_fake_images"},
            update_kwargs={"images": images, "is_real": is_real},
            compute_result=torch.tensor(expected, dtype=torch.float32),
            min_updates_before_compute=2,
            atol=1e-3,
            rtol=1e-3,
        )

    def test_identical_distributions_near_zero(self) -> None:
        torch.manual_seed(5)
        m = FrechetInceptionDistance(model=_Features(8), feature_dim=8)
        x = torch.rand(64, 3, 8, 8)
        m.update(x, True).update(x, False)
        assert abs(float(m.compute())) < 1e-3

    def test_empty_warns(self) -> None:
        m = FrechetInceptionDistance(model=_Features(8), feature_dim=8)
        with pytest.warns(RuntimeWarning, match="Returning 0.0"):
            assert float(m.compute()) == 0.0

    def test_invalid(self) -> None:
        with pytest.raises(RuntimeError, match="feature_dim has to be a positive integer"):
            FrechetInceptionDistance(model=_Features(8), feature_dim=0)
        with pytest.raises(RuntimeError, match="feature_dim needs to be set to 2048"):
            FrechetInceptionDistance(feature_dim=8)
        m = FrechetInceptionDistance(model=_Features(8), feature_dim=8)
        with pytest.raises(ValueError, match="Expected 4D tensor"):
            m.update(torch.rand(3, 8, 8), True)
        with pytest.raises(ValueError, match="Expected 3 channels"):
            m.update(torch.rand(2, 1, 8, 8), True)
        with pytest.raises(ValueError, match="of type bool"):
            m.update(torch.rand(2, 3, 8, 8), 1)

    def test_default_model_validation(self) -> None:
        with pytest.warns(RuntimeWarning, match="randomly initialised"):
            m = FrechetInceptionDistance()
        with pytest.raises(ValueError, match="torch.float32"):
            m.update(torch.rand(2, 3, 32, 32).double(), True)
        with pytest.raises(ValueError, match=r"\[0, 1\] interval"):
            m.update(torch.rand(2, 3, 32, 32) + 1, True)
        m.update(torch.rand(2, 3, 75, 75), True)
        assert int(m.num_real_images) == 2


class TestFIDSingular:
    """Fewer samples than features: S1 has no Cholesky factor, so compute() takes the eigh /
    rank-r path - pinned against scipy's sqrtm oracle."""

    def test_fewer_samples_than_features(self) -> None:
        g = torch.Generator().manual_seed(11)
        for n, d in ((30, 64), (10, 40), (63, 64)):
            real = torch.rand(n, d, generator=g, dtype=torch.float64)
            fake = torch.rand(n + 5, d, generator=g, dtype=torch.float64) ** 2
            m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=d)
            m.update_activations(real.float(), True).update_activations(fake.float(), False)
            want = _fid_oracle(real.float().double().numpy(), fake.float().double().numpy())
            torch.testing.assert_close(m.compute(), torch.tensor(want, dtype=torch.float32), rtol=2e-3, atol=2e-3)

    def test_zero_s1_gives_zero_trace_term(self) -> None:
        from torcheval_amd.metrics.image.fid import _tr_sqrt_product

        s2 = torch.eye(6, dtype=torch.float64)
        assert float(_tr_sqrt_product(torch.zeros(6, 6, dtype=torch.float64), s2)) == 0.0
        # identical real samples: zero covariance, FID = |mu1 - mu2|^2 + tr S2
        m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=6)
        real = torch.ones(5, 6)
        fake = torch.rand(20, 6, generator=torch.Generator().manual_seed(1))
        m.update_activations(real, True).update_activations(fake, False)
        f = fake.double()
        want = (f.mean(0) - 1).square().sum() + torch.cov(f.T).trace()
        torch.testing.assert_close(m.compute(), want.float(), rtol=1e-4, atol=1e-5)

    def test_misaligned_activation_view(self) -> None:
        base = torch.rand(33 * 16 + 1)
        act = base[1:].view(33, 16)  # contiguous, storage offset of one float
        m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=16)
        m.update_activations(act, True)
        torch.testing.assert_close(m.real_cov_sum, act.T @ act, rtol=1e-5, atol=1e-4)
