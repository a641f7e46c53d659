"""K5 deferred mode (metrics/_pending.py): MeanSquaredError / R2Score class updates add FP64
partials to pending slots and the states fold them when read.  Every way a state can be read
or replaced sees exactly the folded sums: compute, direct reads, state_dict / load_state_dict,
merge_state, reset, copies / pickle, to(), a 1-D update after 2-D ones, and HIP-graph replays;
all against fp64 references of reference mean_squared_error.py:82-111 / r2_score.py:97-130."""

import copy
import pickle

import pytest
import torch

from torcheval_amd.metrics import MeanSquaredError, R2Score
from torcheval_amd.metrics.functional import r2_score
from torcheval_amd.metrics.toolkit import sync_and_compute

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _data(n, d, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, d, generator=g), torch.randn(n, d, generator=g) + 1.0


def _sse(xs, ys):
    return sum(((y.double() - x.double()) ** 2).sum(0) for x, y in zip(xs, ys))


def test_pending_then_every_read():
    xs, ys = zip(*[_data(4096, 1001, s) for s in range(3)])
    m = MeanSquaredError(multioutput="raw_values", device=DEV)
    for x, y in zip(xs, ys):
        m.update(x.to(DEV), y.to(DEV))
    assert m.__dict__["_pend_dirty"]  # the updates ran in deferred mode
    ref = _sse(xs, ys)
    torch.testing.assert_close(m.sum_squared_error.cpu().double(), ref, rtol=1e-6, atol=1e-4)
    assert not m.__dict__["_pend_dirty"]
    assert float(m.sum_weight) == 3 * 4096
    torch.testing.assert_close(m.compute().cpu().double(), ref / (3 * 4096), rtol=1e-6, atol=1e-6)
    # more updates after a fold, then state_dict / load_state_dict
    m.update(xs[0].to(DEV), ys[0].to(DEV))
    sd = m.state_dict()
    torch.testing.assert_close(sd["sum_squared_error"].cpu().double(), ref + _sse(xs[:1], ys[:1]), rtol=1e-6, atol=1e-4)
    m2 = MeanSquaredError(multioutput="raw_values", device=DEV)
    m2.update(xs[1].to(DEV), ys[1].to(DEV))  # pending in m2 ...
    m2.load_state_dict(sd)  # ... replaced: the loaded states win for the replaced states
    torch.testing.assert_close(m2.sum_squared_error.cpu(), sd["sum_squared_error"].cpu())


def test_reset_drops_pending_and_copies_fold():
    x, y = _data(2048, 64, 7)
    m = MeanSquaredError(device=DEV)
    m.update(x.to(DEV), y.to(DEV))
    c = copy.deepcopy(m)
    p = pickle.loads(pickle.dumps(m))
    for other in (c, p):
        torch.testing.assert_close(other.sum_squared_error.cpu().double(), _sse([x], [y]), rtol=1e-6, atol=1e-4)
    m.update(x.to(DEV), y.to(DEV))
    m.reset()
    assert float(m.sum_weight) == 0.0 and not bool(m.sum_squared_error.any())
    m.update(x.to(DEV), y.to(DEV))
    torch.testing.assert_close(m.sum_squared_error.cpu().double(), _sse([x], [y]), rtol=1e-6, atol=1e-4)


def test_merge_to_and_mixed_rank_updates():
    xs, ys = zip(*[_data(1500, 17, s) for s in range(4)])
    ms = [MeanSquaredError(multioutput="raw_values", device=DEV) for _ in range(4)]
    for m, x, y in zip(ms, xs, ys):
        m.update(x.to(DEV), y.to(DEV))
    ms[0].merge_state(ms[1:])
    torch.testing.assert_close(ms[0].sum_squared_error.cpu().double(), _sse(xs, ys), rtol=1e-6, atol=1e-4)
    for m, x, y in zip(ms[1:], xs[1:], ys[1:]):  # inputs to merge unchanged
        torch.testing.assert_close(m.sum_squared_error.cpu().double(), _sse([x], [y]), rtol=1e-6, atol=1e-4)
    ms[1].update(xs[0].to(DEV), ys[0].to(DEV))
    cpu = ms[1].to("cpu")
    torch.testing.assert_close(cpu.sum_squared_error.double(), _sse(xs[:2], ys[:2]), rtol=1e-6, atol=1e-4)
    # R2: 2-D deferred updates, then a fold through compute, a sync at ws=1
    r = R2Score(multioutput="raw_values", device=DEV)
    for x, y in zip(xs, ys):
        r.update(x.to(DEV), y.to(DEV))
    ref = r2_score(torch.cat(xs).double(), torch.cat(ys).double(), multioutput="raw_values")
    torch.testing.assert_close(r.compute().cpu().double(), ref, rtol=1e-5, atol=1e-6)
    r.update(xs[0].to(DEV), ys[0].to(DEV))
    ref2 = r2_score(torch.cat(xs + xs[:1]).double(), torch.cat(ys + ys[:1]).double(), multioutput="raw_values")
    torch.testing.assert_close(sync_and_compute(r).cpu().double(), ref2, rtol=1e-5, atol=1e-6)


def test_weighted_and_variable_batches():
    g = torch.Generator().manual_seed(3)
    m = MeanSquaredError(multioutput="raw_values", device=DEV)
    num, den = 0.0, 0.0
    for n in (1, 300, 70001, 5):
        x, y = torch.randn(n, 33, generator=g), torch.randn(n, 33, generator=g)
        w = torch.rand(n, generator=g)
        m.update(x.to(DEV), y.to(DEV), sample_weight=w.to(DEV))
        num = num + (((y.double() - x.double()) ** 2) * w.double()[:, None]).sum(0)
        den += float(w.double().sum())
    torch.testing.assert_close(m.sum_squared_error.cpu().double(), num, rtol=1e-6, atol=1e-4)
    assert float(m.sum_weight) == pytest.approx(den, rel=1e-6)


def test_sum_mean_deferred_long_rows():
    from torcheval_amd.metrics import Mean, Sum

    g = torch.Generator().manual_seed(9)
    s, m = Sum(device=DEV), Mean(device=DEV)
    ref_s, ref_w = 0.0, 0.0
    batches = [(torch.randn(8192, 1001, generator=g), 0.5), (torch.randn(7, generator=g), 2.0),
               (torch.randn(100_003, generator=g), 1.0), (torch.randn(3000, 40, generator=g), "t")]
    for x, w in batches:
        if w == "t":
            wt = torch.rand(x.shape, generator=g)
            s.update(x.to(DEV), weight=wt.to(DEV))
            m.update(x.to(DEV), weight=wt.to(DEV))
            ref_s += float((x.double() * wt.double()).sum())
            ref_w += float(wt.double().sum())
        else:
            s.update(x.to(DEV), weight=w)
            m.update(x.to(DEV), weight=w)
            ref_s += float(x.double().sum()) * w
            ref_w += w * x.numel()
    assert s.__dict__["_pend_dirty"] and m.__dict__["_pend_dirty"]
    assert float(s.compute()) == pytest.approx(ref_s, rel=1e-10, abs=1e-6)
    assert float(m.compute()) == pytest.approx(ref_s / ref_w, rel=1e-10, abs=1e-10)
    # reset drops pending sums; merge / state_dict / copies fold them
    x = torch.randn(50_000, generator=g)
    s.update(x.to(DEV))
    c = copy.deepcopy(s)
    assert float(c.weighted_sum) == pytest.approx(ref_s + float(x.double().sum()), rel=1e-10, abs=1e-6)
    s.reset()
    assert float(s.compute()) == 0.0
    s.update(x.to(DEV))
    s2 = Sum(device=DEV)
    s2.update(x.to(DEV))
    s.merge_state([s2])
    assert float(s.weighted_sum) == pytest.approx(2 * float(x.double().sum()), rel=1e-10, abs=1e-6)
    assert float(s.state_dict()["weighted_sum"]) == pytest.approx(2 * float(x.double().sum()), rel=1e-10, abs=1e-6)


def test_graph_replays_fold_every_replay():
    """a HIP-graph replay of a deferred update adds to the pending slots with
    no Python running, so the fold after it must still cover the captured update's slots."""
    import warnings

    from torcheval_amd.metrics import Mean, Sum
    from torcheval_amd.utils.graphs import GraphedUpdate

    g = torch.Generator().manual_seed(21)
    xs, ys = zip(*[_data(4096, 1001, 30 + s) for s in range(4)])
    m = MeanSquaredError(multioutput="raw_values", device=DEV)
    xd, yd = xs[0].to(DEV), ys[0].to(DEV)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)  # replay-vs-direct speed warning
        step = GraphedUpdate(m, xd, yd)
    assert float(m.sum_weight) == 0.0 and not bool(m.sum_squared_error.any())  # capture restored
    seen_x, seen_y = [], []
    for i in range(6):
        x, y = xs[i % 4], ys[i % 4]
        step(x.to(DEV), y.to(DEV))
        seen_x.append(x)
        seen_y.append(y)
        if i % 2 == 1:  # compute() between replays folds; later replays must fold again
            ref = _sse(seen_x, seen_y) / (4096 * len(seen_x))
            torch.testing.assert_close(m.compute().cpu().double(), ref, rtol=1e-6, atol=1e-6)
    # an eager update of the same metric between replays, then replays again
    m.update(xs[1].to(DEV), ys[1].to(DEV))
    step(xs[2].to(DEV), ys[2].to(DEV))
    seen_x += [xs[1], xs[2]]
    seen_y += [ys[1], ys[2]]
    torch.testing.assert_close(m.sum_squared_error.cpu().double(), _sse(seen_x, seen_y), rtol=1e-6, atol=1e-4)
    assert float(m.sum_weight) == 4096 * len(seen_x)

    # Sum / Mean with a long 1-D batch (K5b deferred mode), compute between replays
    for cls in (Sum, Mean):
        met = cls(device=DEV)
        v = [torch.randn(200_003, generator=g) for _ in range(3)]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            st = GraphedUpdate(met, v[0].to(DEV))
        tot = 0.0
        for i in range(5):
            st(v[i % 3].to(DEV))
            tot += float(v[i % 3].double().sum())
            want = tot if cls is Sum else tot / (200_003 * (i + 1))
            assert float(met.compute()) == pytest.approx(want, rel=1e-9, abs=1e-6)


def test_psnr_ctr_wc_deferred():
    """PSNR (SSE / count / target extrema / data range), CTR and WeightedCalibration on the K5b
    deferred mode: fold on every read against fp64 references (reference psnr.py:68-85,
    click_through_rate.py:53-68, weighted_calibration.py)."""
    from torcheval_amd.metrics import ClickThroughRate, PeakSignalNoiseRatio, WeightedCalibration

    g = torch.Generator().manual_seed(17)
    xs = [torch.rand(64, 3, 33, 35, generator=g) * 2 - 0.3 for _ in range(3)]
    ts = [torch.rand(64, 3, 33, 35, generator=g) * (1.5 + i) - i for i in range(3)]
    for auto in (True, False):
        m = PeakSignalNoiseRatio(data_range=None if auto else 2.0, device=DEV)
        for x, t in zip(xs, ts):
            m.update(x.to(DEV), t.to(DEV))
        assert m.__dict__["_pend_dirty"]
        sse = sum(float(((x.double() - t.double()) ** 2).sum()) for x, t in zip(xs, ts))
        n = sum(x.numel() for x in xs)
        assert float(m.sum_squared_error) == pytest.approx(sse, rel=1e-6)
        assert float(m.num_observations) == n
        if auto:
            lo, hi = min(float(t.min()) for t in ts), max(float(t.max()) for t in ts)
            assert float(m.min_target) == lo and float(m.max_target) == hi
            assert float(m.data_range) == pytest.approx(hi - lo, rel=1e-7)
        rng = (hi - lo) if auto else 2.0
        want = 10 * torch.log10(torch.tensor(rng ** 2 / (sse / n), dtype=torch.float64))
        assert float(m.compute()) == pytest.approx(float(want), rel=1e-5)
        # updates after a fold; a NaN target poisons the range like torch.minimum / maximum
        m.update(xs[0].to(DEV), ts[0].to(DEV))
        assert float(m.num_observations) == n + xs[0].numel()
        bad = ts[1].clone()
        bad[0, 0, 0, 0] = float("nan")
        m.update(xs[1].to(DEV), bad.to(DEV))
        if auto:
            assert torch.isnan(m.min_target.cpu()) and torch.isnan(m.data_range.cpu())
        m.reset()
        assert float(m.num_observations) == 0.0 and float(m.sum_squared_error) == 0.0
        m.update(xs[2].to(DEV), ts[2].to(DEV))
        assert float(m.sum_squared_error) == pytest.approx(float(((xs[2].double() - ts[2].double()) ** 2).sum()), rel=1e-6)

    tasks = 16
    x = [torch.rand(tasks, 40_000, generator=g) for _ in range(2)]
    w = [torch.rand(tasks, 40_000, generator=g) for _ in range(2)]
    t = [torch.rand(tasks, 40_000, generator=g) for _ in range(2)]
    ctr = ClickThroughRate(num_tasks=tasks, device=DEV)
    ctr.update(x[0].to(DEV), w[0].to(DEV))
    ctr.update(x[1].to(DEV), 0.5)
    assert ctr.__dict__["_pend_dirty"]
    clicks = (x[0].double() * w[0].double()).sum(1) + 0.5 * x[1].double().sum(1)
    weights = w[0].double().sum(1) + 0.5 * 40_000
    torch.testing.assert_close(ctr.compute().cpu(), clicks / weights, rtol=1e-10, atol=1e-12)
    wc = WeightedCalibration(num_tasks=tasks, device=DEV)
    wc.update(x[0].to(DEV), t[0].to(DEV), w[0].to(DEV))
    wc.update(x[1].to(DEV), t[1].to(DEV), 2.0)
    num = (x[0].double() * w[0].double()).sum(1) + 2.0 * x[1].double().sum(1)
    den = (t[0].double() * w[0].double()).sum(1) + 2.0 * t[1].double().sum(1)
    torch.testing.assert_close(wc.compute().cpu(), num / den, rtol=1e-10, atol=1e-12)
    # one task, 1-D batches; a state_dict read folds
    c1 = ClickThroughRate(device=DEV)
    c1.update(x[0][0].repeat(3).to(DEV))
    assert float(c1.state_dict()["click_total"][0]) == pytest.approx(3 * float(x[0][0].double().sum()), rel=1e-12)
