"""Aggregation metrics vs numpy oracles (parity: tests/metrics/aggregation/*, functional/aggregation/*)."""

import numpy as np
import pytest
import torch

from torcheval_amd.metrics import AUC, Cat, Max, Mean, Min, Sum, Throughput
from torcheval_amd.metrics.functional import auc, mean, sum as fsum, throughput
from torcheval_amd.utils.test_utils import MetricClassTester


class TestSumMeanMaxMin(MetricClassTester):
    def test_sum(self) -> None:
        x = torch.rand(8, 16)
        self.run_class_implementation_tests(
            metric=Sum(), state_names={"weighted_sum"}, update_kwargs={"input": x},
            compute_result=x.sum().double(), atol=1e-5,
        )

    def test_sum_weighted(self) -> None:
        x, w = torch.rand(8, 16), torch.rand(8, 16)
        self.run_class_implementation_tests(
            metric=Sum(), state_names={"weighted_sum"}, update_kwargs={"input": x, "weight": w},
            compute_result=(x * w).sum().double(), atol=1e-5,
        )

    def test_mean(self) -> None:
        x, w = torch.rand(8, 16), torch.rand(8, 16)
        self.run_class_implementation_tests(
            metric=Mean(), state_names={"weighted_sum", "weights"}, update_kwargs={"input": x, "weight": w},
            compute_result=((x * w).sum() / w.sum()).double(), atol=1e-5,
        )

    def test_max_min(self) -> None:
        x = torch.randn(8, 16)
        self.run_class_implementation_tests(
            metric=Max(), state_names={"max"}, update_kwargs={"input": x}, compute_result=x.max(),
        )
        self.run_class_implementation_tests(
            metric=Min(), state_names={"min"}, update_kwargs={"input": x}, compute_result=x.min(),
        )

    def test_cat(self) -> None:
        x = torch.randn(8, 4, 3)
        self.run_class_implementation_tests(
            metric=Cat(dim=0), state_names={"dim", "inputs"}, update_kwargs={"input": x},
            compute_result=x.reshape(32, 3),
        )

    def test_functional(self) -> None:
        x, w = torch.rand(10), torch.rand(10)
        torch.testing.assert_close(fsum(x, w), (x * w).sum())
        torch.testing.assert_close(mean(x, w), (x * w).sum() / w.sum())
        torch.testing.assert_close(mean(x, 2.0), x.mean())
        torch.testing.assert_close(throughput(100, 4.0), torch.tensor(25.0))
        with pytest.raises(ValueError):
            throughput(-1, 1.0)
        with pytest.raises(ValueError):
            throughput(1, 0.0)


class TestAUC(MetricClassTester):
    def test_functional_vs_numpy(self) -> None:
        torch.manual_seed(0)
        x = torch.rand(50).sort().values
        y = torch.rand(50)
        torch.testing.assert_close(auc(x, y), torch.tensor([np.trapz(y.numpy(), x.numpy())], dtype=torch.float32), rtol=1e-5, atol=1e-6)
        perm = torch.randperm(50)
        torch.testing.assert_close(auc(x[perm], y[perm], reorder=True), auc(x, y), rtol=1e-5, atol=1e-6)

    def test_class(self) -> None:
        torch.manual_seed(1)
        x, y = torch.rand(8, 10), torch.rand(8, 10)
        fx, fy = x.flatten(), y.flatten()
        order = fx.argsort()
        expected = torch.tensor(np.trapz(fy[order].numpy(), fx[order].numpy()), dtype=torch.float32)
        self.run_class_implementation_tests(
            metric=AUC(), state_names={"x", "y"}, update_kwargs={"x": x, "y": y},
            compute_result=expected.reshape(1), atol=1e-5,
        )


class TestThroughput(MetricClassTester):
    def test_class(self) -> None:
        m = Throughput()
        m.update(100, 2.0).update(50, 1.0)
        assert m.compute() == pytest.approx(50.0)
        m2 = Throughput().update(30, 3.0)
        m.merge_state([m2])
        # merged: total items / max elapsed (ranks run concurrently)
        assert m.compute() == pytest.approx(180 / 3.0)
        with pytest.raises(ValueError):
            Throughput().update(-1, 1.0)
