"""K5b (csrc/kernels/rowsums.hip): fused per-row weighted sums merged into metric states, on
the GPU, against FP64 ATen references of the same updates (the reference's op chains)."""

import pytest
import torch

from torcheval_amd.metrics import (
    ClickThroughRate,
    Mean,
    MeanSquaredError,
    PeakSignalNoiseRatio,
    R2Score,
    Sum,
    WeightedCalibration,
    WindowedClickThroughRate,
    WindowedWeightedCalibration,
)
from torcheval_amd.metrics.functional import (
    click_through_rate,
    mean,
    peak_signal_noise_ratio,
    sum as fsum,
    weighted_calibration,
)
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
SIZES = [1, 7, 4099, 65536, 65537, 1_000_003, 8192 * 1000]


def _close(got, want, rtol=1e-6, atol=1e-6):
    want = want.double()
    if want.numel() == got.numel():
        want = want.reshape(got.shape)  # 1-task states are [1]
    torch.testing.assert_close(got.cpu().double(), want, rtol=rtol, atol=atol, equal_nan=True)


@pytest.mark.parametrize("n", SIZES)
def test_sum_mean_classes(n):
    g = torch.Generator().manual_seed(n % 1000)
    xs = [torch.rand(n, generator=g) for _ in range(3)]
    ws = [torch.rand(n, generator=g) for _ in range(3)]
    s, m, mw = Sum(device=DEV), Mean(device=DEV), Mean(device=DEV)
    for x, w in zip(xs, ws):
        s.update(x.to(DEV))
        m.update(x.to(DEV), weight=0.5)
        mw.update(x.to(DEV), weight=w.to(DEV))
    X, W = torch.cat(xs).double(), torch.cat(ws).double()
    _close(s.compute(), X.sum(), rtol=1e-9)
    _close(m.compute(), X.mean(), rtol=1e-9)
    _close(mw.compute(), (W * X).sum() / W.sum(), rtol=1e-9)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.uint8])
def test_sum_mean_dtypes_and_strides(dtype):
    g = torch.Generator().manual_seed(1)
    base = (torch.rand(300, 40, generator=g) * 10).to(dtype)
    x = base.t()  # non-contiguous: the generic (strided) load path
    s = Sum(device=DEV).update(x.to(DEV))
    _close(s.compute(), x.double().sum(), rtol=1e-6)
    m = Mean(device=DEV).update(x.to(DEV), weight=3)
    _close(m.compute(), x.double().mean(), rtol=1e-6)


@pytest.mark.parametrize("n", [5, 10_000, 200_001])
def test_functional_sum_mean(n):
    g = torch.Generator().manual_seed(n)
    x, w = torch.randn(n, generator=g), torch.rand(n, generator=g)
    _close(fsum(x.to(DEV)), x.double().sum(), rtol=1e-5, atol=1e-4)
    _close(fsum(x.to(DEV), w.to(DEV)), (x.double() * w.double()).sum(), rtol=1e-5, atol=1e-4)
    _close(mean(x.to(DEV), w.to(DEV)), (x.double() * w.double()).sum() / w.double().sum(), rtol=1e-5, atol=1e-5)
    assert fsum(x.to(DEV)).dtype == torch.float32 and mean(x.double().to(DEV)).dtype == torch.float64


@pytest.mark.parametrize("tasks,n", [(1, 9), (1, 300_000), (4, 8192), (32, 70_000)])
def test_ctr_wc_classes(tasks, n):
    g = torch.Generator().manual_seed(tasks * n)
    shape = (n,) if tasks == 1 else (tasks, n)
    c = ClickThroughRate(num_tasks=tasks, device=DEV)
    wc = WeightedCalibration(num_tasks=tasks, device=DEV)
    wcc = WindowedClickThroughRate(num_tasks=tasks, max_num_updates=2, device=DEV)
    wwc = WindowedWeightedCalibration(num_tasks=tasks, max_num_updates=2, device=DEV)
    batches = []
    for _ in range(3):
        clicks = (torch.rand(shape, generator=g) < 0.3).float()
        w = torch.rand(shape, generator=g)
        x, t = torch.rand(shape, generator=g), (torch.rand(shape, generator=g) < 0.5).float()
        c.update(clicks.to(DEV), w.to(DEV))
        wc.update(x.to(DEV), t.to(DEV), w.to(DEV))
        wcc.update(clicks.to(DEV), w.to(DEV))
        wwc.update(x.to(DEV), t.to(DEV))
        batches.append((clicks.double(), w.double(), x.double(), t.double()))
    C = torch.cat([b[0] for b in batches], -1)
    W = torch.cat([b[1] for b in batches], -1)
    X = torch.cat([b[2] for b in batches], -1)
    T = torch.cat([b[3] for b in batches], -1)
    _close(c.compute(), (C * W).sum(-1) / W.sum(-1), rtol=1e-9)
    _close(wc.compute(), (W * X).sum(-1) / (W * T).sum(-1), rtol=1e-9)
    life, win = wcc.compute()
    _close(life, (C * W).sum(-1) / W.sum(-1), rtol=1e-9)
    cw = torch.cat([b[0] * b[1] for b in batches[1:]], -1).sum(-1)
    ww = torch.cat([b[1] for b in batches[1:]], -1).sum(-1)
    _close(win, cw / ww, rtol=1e-9)
    life, win = wwc.compute()
    _close(life, X.sum(-1) / T.sum(-1), rtol=1e-9)
    xw = torch.cat([b[2] for b in batches[1:]], -1).sum(-1)
    tw = torch.cat([b[3] for b in batches[1:]], -1).sum(-1)
    _close(win, xw / tw, rtol=1e-9)


def test_ctr_wc_functional():
    g = torch.Generator().manual_seed(3)
    clicks = (torch.rand(3, 5000, generator=g) < 0.2).float()
    w = torch.rand(3, 5000, generator=g)
    got = click_through_rate(clicks.to(DEV), w.to(DEV), num_tasks=3)
    _close(got, click_through_rate(clicks, w, num_tasks=3), rtol=1e-5)
    got = click_through_rate(clicks[0].to(DEV))
    _close(got, click_through_rate(clicks[0]), rtol=1e-6)
    x, t = torch.rand(3, 5000, generator=g), torch.rand(3, 5000, generator=g)
    _close(weighted_calibration(x.to(DEV), t.to(DEV), w.to(DEV), num_tasks=3),
           weighted_calibration(x, t, w, num_tasks=3), rtol=1e-5)


@pytest.mark.parametrize("auto", [True, False])
@pytest.mark.parametrize("shape", [(2, 3, 4, 4), (16, 3, 64, 64), (8, 3, 256, 256)])
def test_psnr(auto, shape):
    g = torch.Generator().manual_seed(sum(shape))
    m = PeakSignalNoiseRatio(data_range=None if auto else 1.0, device=DEV)
    ref = PeakSignalNoiseRatio(data_range=None if auto else 1.0)
    for k in range(3):
        x, t = torch.rand(shape, generator=g), torch.rand(shape, generator=g) * (1 + k)
        m.update(x.to(DEV), t.to(DEV))
        ref.update(x.double(), t.double())
    _close(m.compute(), ref.compute(), rtol=1e-5, atol=1e-5)
    _close(m.data_range, ref.data_range, rtol=1e-6)
    x, t = torch.rand(shape, generator=g), torch.rand(shape, generator=g)
    _close(peak_signal_noise_ratio(x.to(DEV), t.to(DEV)), peak_signal_noise_ratio(x.double(), t.double()), rtol=1e-5)
    _close(peak_signal_noise_ratio(x.to(DEV), t.to(DEV), data_range=2.0),
           peak_signal_noise_ratio(x.double(), t.double(), data_range=2.0), rtol=1e-5)


def test_psnr_nan_target_propagates():
    t = torch.rand(4, 3, 8, 8)
    t[1, 2, 3, 4] = float("nan")
    m = PeakSignalNoiseRatio(device=DEV).update(torch.rand(4, 3, 8, 8).to(DEV), t.to(DEV))
    assert torch.isnan(m.max_target.cpu()) and torch.isnan(m.min_target.cpu())


@pytest.mark.parametrize("shape", [(8,), (1000,), (8192, 1000), (100_000, 3)])
@pytest.mark.parametrize("weighted", [False, True])
def test_mse_r2_classes(shape, weighted):
    g = torch.Generator().manual_seed(len(shape) + shape[0])
    m, r = MeanSquaredError(multioutput="raw_values", device=DEV), R2Score(multioutput="raw_values", device=DEV)
    xs, ts, ws = [], [], []
    for _ in range(2):
        x, t = torch.rand(shape, generator=g), torch.rand(shape, generator=g)
        w = torch.rand(shape[0], generator=g) if weighted else None
        m.update(x.to(DEV), t.to(DEV), sample_weight=None if w is None else w.to(DEV))
        r.update(x.to(DEV), t.to(DEV))
        xs.append(x.double()), ts.append(t.double()), ws.append(w)
    X, T = torch.cat(xs), torch.cat(ts)
    Wt = torch.cat(ws).double() if weighted else torch.ones(X.shape[0], dtype=torch.float64)
    Wb = Wt[:, None] if X.ndim == 2 else Wt
    _close(m.compute(), ((X - T) ** 2 * Wb).sum(0) / Wt.sum(), rtol=1e-5, atol=1e-6)
    tss = ((T - T.mean(0)) ** 2).sum(0)
    _close(r.compute(), 1 - ((X - T) ** 2).sum(0) / tss, rtol=1e-4, atol=1e-5)


def test_row_sums_raw_ops():
    """Direct K5b call: every stat with SET / ADD / MIN / MAX into f32 and f64 outputs,
    strided ring-slot outputs and row-0-only scalars."""
    from torcheval_amd.ops import rowsums as rs

    g = torch.Generator().manual_seed(0)
    x, t, w = (torch.randn(5, 70_000, generator=g) for _ in range(3))
    ring = torch.zeros(5, 4, dtype=torch.float64, device=DEV)
    acc = torch.full((5,), 2.0, device=DEV)
    mn = torch.full((5,), 0.0, dtype=torch.float64, device=DEV)
    mx = torch.full((5,), 0.0, device=DEV)
    cnt = torch.zeros((), device=DEV)
    rs.update_states(x.to(DEV), t.to(DEV), w.to(DEV), [
        (ring[:, 2], rs.WX, rs.SET), (acc, rs.WSSE, rs.ADD), (mn, rs.TMIN, rs.MIN), (mx, rs.TMAX, rs.MAX),
        (cnt, rs.COUNT, rs.ADD | rs.FIRST_ROW)], rows=5)
    X, T, W = x.double(), t.double(), w.double()
    _close(ring[:, 2], (W * X).sum(-1), rtol=1e-9)
    assert float(ring[:, [0, 1, 3]].abs().sum()) == 0.0
    _close(acc, 2.0 + (W * (X - T) ** 2).sum(-1), rtol=1e-6)
    _close(mn, torch.minimum(T.min(-1).values, torch.zeros(5, dtype=torch.float64)), rtol=0, atol=0)
    _close(mx, torch.maximum(T.max(-1).values.float().double(), torch.zeros(5, dtype=torch.float64)), rtol=0, atol=0)
    assert float(cnt) == 70_000.0
    assert native() is not None
