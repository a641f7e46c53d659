"""Ranking metrics vs brute-force loops (parity: tests/metrics/ranking/*, functional/ranking/*)."""

import pytest
import torch

from torcheval_amd.metrics import ClickThroughRate, HitRate, ReciprocalRank, RetrievalPrecision, WeightedCalibration
from torcheval_amd.metrics.functional import (
    click_through_rate,
    frequency_at_k,
    hit_rate,
    num_collisions,
    reciprocal_rank,
    retrieval_precision,
    weighted_calibration,
)
from torcheval_amd.utils.test_utils import MetricClassTester


def _rank(row: torch.Tensor, t: int) -> int:
    return int((row > row[t]).sum())


def _hit_oracle(x, y, k):
    return torch.tensor([float(_rank(r, int(t)) < (k if k is not None else r.numel())) for r, t in zip(x, y)])


def _rr_oracle(x, y, k):
    out = []
    for r, t in zip(x, y):
        rk = _rank(r, int(t))
        out.append(0.0 if (k is not None and rk >= k) else 1.0 / (rk + 1))
    return torch.tensor(out)


class TestRankingFunctional:
    def test_hit_rate_and_rr(self) -> None:
        torch.manual_seed(0)
        x = torch.randint(0, 6, (30, 7)).float()  # heavy ties
        y = torch.randint(0, 7, (30,))
        for k in (None, 1, 3, 7):
            torch.testing.assert_close(hit_rate(x, y, k=k), _hit_oracle(x, y, k))
            torch.testing.assert_close(reciprocal_rank(x, y, k=k), _rr_oracle(x, y, k))
        with pytest.raises(ValueError):
            hit_rate(x, y, k=0)
        with pytest.raises(ValueError):
            hit_rate(x[0], y)

    def test_num_collisions_frequency(self) -> None:
        x = torch.tensor([3, 4, 2, 3, 3, 9, 4])
        torch.testing.assert_close(num_collisions(x), torch.tensor([2, 1, 0, 2, 2, 0, 1]))
        f = torch.tensor([0.3, 0.1, 0.6, 2.0])
        torch.testing.assert_close(frequency_at_k(f, 0.5), torch.tensor([1.0, 1.0, 0.0, 0.0]))
        with pytest.raises(ValueError):
            frequency_at_k(f, -1)

    def test_ctr_and_calibration(self) -> None:
        x = torch.tensor([[1, 0, 0, 1], [1, 1, 1, 1]])
        w = torch.tensor([[1.0, 2.0, 3.0, 4.0], [0.5, 0.5, 0.5, 0.5]])
        torch.testing.assert_close(click_through_rate(x, w, num_tasks=2), torch.tensor([0.5, 1.0]))
        torch.testing.assert_close(click_through_rate(torch.tensor([1, 0, 1, 1])), torch.tensor(0.75))
        p, t = torch.tensor([0.2, 0.6, 0.7]), torch.tensor([0.0, 1.0, 1.0])
        torch.testing.assert_close(weighted_calibration(p, t), torch.tensor(1.5 / 2.0, dtype=p.dtype))
        with pytest.raises(ValueError):
            click_through_rate(x, num_tasks=3)

    def test_retrieval_precision(self) -> None:
        x = torch.tensor([0.5, 0.9, 0.1, 0.7, 0.3])
        t = torch.tensor([1, 0, 0, 1, 1])
        # top-3 by score: 0.9(0), 0.7(1), 0.5(1)
        torch.testing.assert_close(retrieval_precision(x, t, k=3), torch.tensor(2 / 3))
        torch.testing.assert_close(retrieval_precision(x, t, k=10), torch.tensor(3 / 10))
        torch.testing.assert_close(retrieval_precision(x, t, k=10, limit_k_to_size=True), torch.tensor(3 / 5))
        with pytest.raises(ValueError):
            retrieval_precision(x, t, k=0)


class TestRankingClasses(MetricClassTester):
    def test_hit_rate_and_rr_class(self) -> None:
        torch.manual_seed(1)
        x = torch.rand(8, 6, 10)
        y = torch.randint(0, 10, (8, 6))
        fx, fy = x.reshape(-1, 10), y.flatten()
        self.run_class_implementation_tests(
            metric=HitRate(k=3), state_names={"scores"}, update_kwargs={"input": x, "target": y},
            compute_result=_hit_oracle(fx, fy, 3),
        )
        self.run_class_implementation_tests(
            metric=ReciprocalRank(), state_names={"scores"}, update_kwargs={"input": x, "target": y},
            compute_result=_rr_oracle(fx, fy, None),
        )

    def test_ctr_class(self) -> None:
        torch.manual_seed(2)
        x, w = torch.randint(0, 2, (8, 2, 12)), torch.rand(8, 2, 12)
        fx, fw = x.permute(1, 0, 2).reshape(2, -1), w.permute(1, 0, 2).reshape(2, -1)
        self.run_class_implementation_tests(
            metric=ClickThroughRate(num_tasks=2), state_names={"click_total", "weight_total"},
            update_kwargs={"input": x, "weights": w},
            compute_result=((fx * fw).sum(-1) / fw.sum(-1)).double(), atol=1e-6,
        )

    def test_weighted_calibration_class(self) -> None:
        torch.manual_seed(3)
        x, t = torch.rand(8, 12), torch.randint(0, 2, (8, 12)).float()
        self.run_class_implementation_tests(
            metric=WeightedCalibration(), state_names={"weighted_input_sum", "weighted_target_sum"},
            update_kwargs={"input": x, "target": t},
            compute_result=(x.sum() / t.sum()).double().reshape(1), atol=1e-6,
        )

    def test_retrieval_precision_class(self) -> None:
        torch.manual_seed(4)
        x, t = torch.rand(8, 10), torch.randint(0, 2, (8, 10))
        fx, ft = x.flatten(), t.flatten()
        self.run_class_implementation_tests(
            metric=RetrievalPrecision(k=5), state_names={"topk", "target", "count"},
            update_kwargs={"input": x, "target": t},
            compute_result=retrieval_precision(fx, ft, k=5).reshape(1),
        )

    def test_retrieval_precision_queries(self) -> None:
        m = RetrievalPrecision(k=2, num_queries=3, empty_target_action="skip")
        m.update(torch.tensor([0.9, 0.1, 0.8, 0.4]), torch.tensor([1, 0, 0, 0]), indexes=torch.tensor([0, 0, 1, 1]))
        m.update(torch.tensor([0.7, 0.95]), torch.tensor([1, 1]), indexes=torch.tensor([0, 1]))
        out = m.compute()
        # query 0 top-2: 0.9(1), 0.7(1) -> 1.0; query 1 top-2: 0.95(1), 0.8(0) -> 0.5; query 2 empty -> nan
        torch.testing.assert_close(out[:2], torch.tensor([1.0, 0.5]))
        assert torch.isnan(out[2])
        with pytest.raises(ValueError, match="no positive value found"):
            RetrievalPrecision(empty_target_action="err").update(torch.rand(3), torch.zeros(3)).compute()


def _rp_oracle(batches, k, num_queries, limit_k_to_size, action):
    """The reference's algorithm: per-query lists of streaming top-k, then precision@k."""
    tops = [(torch.empty(0), torch.empty(0)) for _ in range(num_queries)]
    for x, t, idx in batches:
        for i in range(num_queries):
            sel = idx == i
            if not bool(sel.any()):
                continue
            v = torch.cat([tops[i][0], x[sel]])
            tt = torch.cat([tops[i][1], t[sel].float()])
            kk = v.numel() if k is None else min(k, v.numel())
            vv, j = v.topk(kk)
            tops[i] = (vv, tt[j])
    out = []
    for v, t in tops:
        if not len(t):
            out.append(float("nan"))
        elif not bool((t == 1).any()):
            out.append({"pos": 1.0, "neg": 0.0, "skip": float("nan")}[action])
        else:
            total = v.numel() if k is None else (min(k, v.numel()) if limit_k_to_size else k)
            out.append(float(t.sum()) / total)
    return torch.tensor(out)


@pytest.mark.parametrize("k", [None, 1, 3, 7])
@pytest.mark.parametrize("limit", [False, True])
@pytest.mark.parametrize("action", ["neg", "pos", "skip"])
def test_retrieval_precision_dense_state_matches_oracle(k, limit, action):
    if limit and k is None:
        return
    g = torch.Generator().manual_seed((k or 0) * 7 + int(limit))
    Q = 6
    m = RetrievalPrecision(k=k, limit_k_to_size=limit, num_queries=Q, empty_target_action=action)
    batches = []
    for n in (13, 0, 40, 5):
        x = (torch.randint(0, 20, (n,), generator=g) / 20.0)
        t = torch.randint(0, 2, (n,), generator=g)
        idx = torch.randint(-1, Q, (n,), generator=g)  # -1: ignored
        idx[idx == 4] = 5  # query 4 never appears
        m.update(x, t, indexes=idx)
        batches.append((x, t, idx))
    want = _rp_oracle(batches, k, Q, limit, action)
    torch.testing.assert_close(m.compute(), want, equal_nan=True)
    # merge two halves == one metric over everything
    a = RetrievalPrecision(k=k, limit_k_to_size=limit, num_queries=Q, empty_target_action=action)
    b = RetrievalPrecision(k=k, limit_k_to_size=limit, num_queries=Q, empty_target_action=action)
    for x, t, idx in batches[:2]:
        a.update(x, t, indexes=idx)
    for x, t, idx in batches[2:]:
        b.update(x, t, indexes=idx)
    torch.testing.assert_close(a.merge_state([b]).compute(), want, equal_nan=True)


def test_retrieval_precision_loads_reference_state_dict():
    ref_sd = {"topk": [torch.tensor([0.9, 0.5]), torch.empty(0)], "target": [torch.tensor([1.0, 0.0]), torch.empty(0)]}
    m = RetrievalPrecision(k=2, num_queries=2)
    m.load_state_dict(ref_sd)
    out = m.compute()
    torch.testing.assert_close(out[0], torch.tensor(0.5))
    assert torch.isnan(out[1])
