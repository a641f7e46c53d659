"""Windowed metrics: reference docstring/test values + brute-force window oracles
(parity: tests/metrics/window/*.py)."""

import pytest
import torch

from torcheval_amd.metrics import (
    BinaryAUROC,
    ClickThroughRate,
    WindowedBinaryAUROC,
    WindowedBinaryNormalizedEntropy,
    WindowedClickThroughRate,
    WindowedMeanSquaredError,
    WindowedWeightedCalibration,
)
from torcheval_amd.metrics.functional import (
    binary_auroc,
    binary_normalized_entropy,
    click_through_rate,
    mean_squared_error,
    weighted_calibration,
)
from torcheval_amd.utils.test_utils import MetricClassTester

F64 = torch.float64


class TestWindowedClickThroughRate(MetricClassTester):
    def test_single_task(self) -> None:
        input = torch.tensor([[1, 0, 0, 1], [0, 0, 0, 0], [1, 1, 1, 1], [0, 1, 1, 1]])
        names = {"max_num_updates", "total_updates", "windowed_click_total", "windowed_weight_total"}
        self.run_class_implementation_tests(
            metric=WindowedClickThroughRate(num_tasks=1, max_num_updates=2, enable_lifetime=True),
            state_names=names | {"click_total", "weight_total"},
            update_kwargs={"input": input},
            compute_result=(torch.tensor([0.5625], dtype=F64), torch.tensor([0.875], dtype=F64)),
            merge_and_compute_result=(torch.tensor([0.5625], dtype=F64), torch.tensor([0.5625], dtype=F64)),
            num_total_updates=4,
            num_processes=2,
        )
        self.run_class_implementation_tests(
            metric=WindowedClickThroughRate(num_tasks=1, max_num_updates=2, enable_lifetime=False),
            state_names=names,
            update_kwargs={"input": input},
            compute_result=torch.tensor([0.875], dtype=F64),
            merge_and_compute_result=torch.tensor([0.5625], dtype=F64),
            num_total_updates=4,
            num_processes=2,
        )

    def test_multi_task_weighted(self) -> None:
        input = torch.tensor(
            [[[1, 0, 0, 1], [1, 1, 1, 1]], [[0, 0, 0, 0], [1, 1, 1, 1]],
             [[0, 1, 0, 1], [0, 1, 0, 1]], [[1, 1, 1, 1], [0, 1, 1, 1]]]
        )
        weights = torch.tensor(
            [[[1, 2, 3, 4], [0, 0, 0, 0]], [[1, 2, 1, 2], [1, 2, 1, 2]],
             [[1, 1, 1, 1], [1, 1, 3, 1]], [[1, 1, 1, 1], [1, 1, 1, 1]]]
        )
        life = click_through_rate(input.permute(1, 0, 2).reshape(2, -1), weights.permute(1, 0, 2).reshape(2, -1), num_tasks=2)
        win = click_through_rate(input[2:].permute(1, 0, 2).reshape(2, -1), weights[2:].permute(1, 0, 2).reshape(2, -1), num_tasks=2)
        self.run_class_implementation_tests(
            metric=WindowedClickThroughRate(num_tasks=2, max_num_updates=2),
            state_names={"max_num_updates", "total_updates", "click_total", "weight_total",
                         "windowed_click_total", "windowed_weight_total"},
            update_kwargs={"input": input, "weights": weights},
            compute_result=(life.double(), win.double()),
            merge_and_compute_result=(life.double(), life.double()),
            num_total_updates=4,
            num_processes=2,
        )

    def test_ring_against_bruteforce(self) -> None:
        torch.manual_seed(0)
        m = WindowedClickThroughRate(max_num_updates=3)
        hist = []
        for _ in range(7):
            x = torch.randint(0, 2, (10,))
            m.update(x)
            hist.append(x)
            life, win = m.compute()
            torch.testing.assert_close(life, click_through_rate(torch.cat(hist)).double().reshape(1))
            torch.testing.assert_close(win, click_through_rate(torch.cat(hist[-3:])).double().reshape(1))

    def test_invalid(self) -> None:
        with pytest.raises(ValueError, match="`num_tasks` value should be greater than and equal to 1"):
            WindowedClickThroughRate(num_tasks=0)
        with pytest.raises(ValueError, match="`max_num_updates` value should be greater than and equal to 1"):
            WindowedClickThroughRate(max_num_updates=0)
        assert WindowedClickThroughRate().compute()[0].numel() == 0
        assert WindowedClickThroughRate(enable_lifetime=False).compute().numel() == 0


class TestWindowedNormalizedEntropy(MetricClassTester):
    def test_docstring_values(self) -> None:
        m = WindowedBinaryNormalizedEntropy(max_num_updates=2)
        m.update(torch.tensor([0.2, 0.3]), torch.tensor([1.0, 0.0]))
        m.update(torch.tensor([0.5, 0.6]), torch.tensor([1.0, 1.0]))
        m.update(torch.tensor([0.6, 0.2]), torch.tensor([0.0, 1.0]))
        life, win = m.compute()
        torch.testing.assert_close(life, torch.tensor([1.4914], dtype=F64), atol=1e-4, rtol=0)
        torch.testing.assert_close(win, torch.tensor([1.6581], dtype=F64), atol=1e-4, rtol=0)
        m = WindowedBinaryNormalizedEntropy(max_num_updates=2, num_tasks=2)
        m.update(torch.tensor([[0.2, 0.3], [0.5, 0.1]]), torch.tensor([[1.0, 0.0], [0.0, 1.0]]))
        m.update(torch.tensor([[0.8, 0.3], [0.6, 0.1]]), torch.tensor([[1.0, 1.0], [1.0, 0.0]]))
        m.update(torch.tensor([[0.5, 0.1], [0.3, 0.9]]), torch.tensor([[0.0, 1.0], [0.0, 0.0]]))
        life, win = m.compute()
        torch.testing.assert_close(life, torch.tensor([1.6729, 1.6421], dtype=F64), atol=1e-4, rtol=0)
        torch.testing.assert_close(win, torch.tensor([1.9663, 1.4562], dtype=F64), atol=1e-4, rtol=0)

    def test_class_suite(self) -> None:
        torch.manual_seed(3)
        input = torch.rand(8, 2, 16)
        target = torch.randint(0, 2, (8, 2, 16)).float()
        flat = lambda t: t.permute(1, 0, 2).reshape(2, -1)  # noqa: E731
        life = binary_normalized_entropy(flat(input), flat(target), num_tasks=2)
        win = binary_normalized_entropy(flat(input[-3:]), flat(target[-3:]), num_tasks=2)
        self.run_class_implementation_tests(
            metric=WindowedBinaryNormalizedEntropy(num_tasks=2, max_num_updates=3),
            state_names={"max_num_updates", "total_updates", "total_entropy", "num_examples",
                         "num_positive", "windowed_total_entropy", "windowed_num_examples",
                         "windowed_num_positive"},
            update_kwargs={"input": input, "target": target},
            compute_result=(life, win),
            # 4 ranks x 2 updates each, every rank's 2 updates fit its 3-wide window
            merge_and_compute_result=(life, life),
            num_total_updates=8,
            num_processes=4,
        )

    def test_logits_and_weight(self) -> None:
        torch.manual_seed(4)
        m = WindowedBinaryNormalizedEntropy(from_logits=True, max_num_updates=2, enable_lifetime=False)
        xs, ts, ws = [], [], []
        for _ in range(4):
            x, t, w = torch.randn(12), torch.randint(0, 2, (12,)).float(), torch.rand(12)
            m.update(x, t, weight=w)
            xs.append(x), ts.append(t), ws.append(w)
        expect = binary_normalized_entropy(torch.cat(xs[-2:]), torch.cat(ts[-2:]), weight=torch.cat(ws[-2:]), from_logits=True)
        torch.testing.assert_close(m.compute(), expect.reshape(1), rtol=1e-5, atol=1e-6)


class TestWindowedMeanSquaredError(MetricClassTester):
    def test_class_suite(self) -> None:
        torch.manual_seed(5)
        input, target = torch.rand(8, 16), torch.rand(8, 16)
        life = mean_squared_error(input.flatten(), target.flatten())
        win = mean_squared_error(input[-2:].flatten(), target[-2:].flatten())
        self.run_class_implementation_tests(
            metric=WindowedMeanSquaredError(max_num_updates=2),
            state_names={"max_num_updates", "total_updates", "sum_squared_error", "sum_weight",
                         "windowed_sum_squared_error", "windowed_sum_weight"},
            update_kwargs={"input": input, "target": target},
            compute_result=(life, win),
            merge_and_compute_result=(life, life),
            num_total_updates=8,
            num_processes=4,
            atol=1e-6,
        )

    def test_multioutput_and_weights(self) -> None:
        torch.manual_seed(6)
        m = WindowedMeanSquaredError(num_tasks=3, max_num_updates=2, multioutput="raw_values")
        xs, ts, ws = [], [], []
        for _ in range(5):
            x, t, w = torch.rand(10, 3), torch.rand(10, 3), torch.rand(10)
            m.update(x, t, sample_weight=w)
            xs.append(x), ts.append(t), ws.append(w)
        life, win = m.compute()
        torch.testing.assert_close(life, mean_squared_error(torch.cat(xs), torch.cat(ts), sample_weight=torch.cat(ws), multioutput="raw_values"))
        torch.testing.assert_close(win, mean_squared_error(torch.cat(xs[-2:]), torch.cat(ts[-2:]), sample_weight=torch.cat(ws[-2:]), multioutput="raw_values"))
        with pytest.raises(ValueError, match="expected to be one-dimensional"):
            WindowedMeanSquaredError().update(torch.rand(4, 2), torch.rand(4, 2))
        with pytest.raises(ValueError, match=r"shape is expected to be \(num_samples, 3\)"):
            WindowedMeanSquaredError(num_tasks=3).update(torch.rand(4, 2), torch.rand(4, 2))


class TestWindowedWeightedCalibration(MetricClassTester):
    def test_class_suite(self) -> None:
        torch.manual_seed(7)
        input, target = torch.rand(8, 2, 16), torch.randint(0, 2, (8, 2, 16)).double()
        flat = lambda t: t.permute(1, 0, 2).reshape(2, -1)  # noqa: E731
        life = weighted_calibration(flat(input), flat(target), num_tasks=2)
        win = weighted_calibration(flat(input[-4:]), flat(target[-4:]), num_tasks=2)
        self.run_class_implementation_tests(
            metric=WindowedWeightedCalibration(num_tasks=2, max_num_updates=4),
            state_names={"max_num_updates", "total_updates", "weighted_input_sum", "weighted_target_sum",
                         "windowed_weighted_input_sum", "windowed_weighted_target_sum"},
            update_kwargs={"input": input, "target": target},
            compute_result=(life, win),
            merge_and_compute_result=(life, life),
            num_total_updates=8,
            num_processes=4,
        )


class TestWindowedBinaryAUROC(MetricClassTester):
    def test_docstring_values(self) -> None:
        m = WindowedBinaryAUROC(max_num_samples=4)
        m.update(torch.tensor([0.2, 0.5, 0.1, 0.5, 0.7, 0.8]), torch.tensor([0, 1, 1, 0, 1, 1]))
        torch.testing.assert_close(m.inputs, torch.tensor([[0.1, 0.5, 0.7, 0.8]]))
        torch.testing.assert_close(m.targets, torch.tensor([[1.0, 0.0, 1.0, 1.0]]))
        torch.testing.assert_close(m.compute(), torch.tensor(2 / 3, dtype=F64))
        m = WindowedBinaryAUROC(max_num_samples=5, num_tasks=2)
        m.update(torch.tensor([[0.2, 0.3], [0.5, 0.1]]), torch.tensor([[1.0, 0.0], [0.0, 1.0]]))
        m.update(torch.tensor([[0.8, 0.3], [0.6, 0.1]]), torch.tensor([[1.0, 1.0], [1.0, 0.0]]))
        m.update(torch.tensor([[0.5, 0.1], [0.3, 0.9]]), torch.tensor([[0.0, 1.0], [0.0, 0.0]]))
        torch.testing.assert_close(
            m.inputs, torch.tensor([[0.1, 0.3, 0.8, 0.3, 0.5], [0.9, 0.1, 0.6, 0.1, 0.3]])
        )
        # task 0 matches the reference docstring (0.4167); task 1 is the tie-aware pair count
        # (positives {0.6, 0.1} vs negatives {0.9, 0.1, 0.3}: 2.5 / 6) - the reference
        # docstring's 0.5 predates its tie handling.
        torch.testing.assert_close(m.compute(), torch.tensor([2.5 / 6, 2.5 / 6], dtype=F64), atol=1e-4, rtol=0)

    def test_ring_against_bruteforce(self) -> None:
        torch.manual_seed(8)
        m = WindowedBinaryAUROC(max_num_samples=20)
        xs, ts = [], []
        for n in (7, 9, 3, 25, 11, 0, 4):
            x, t = torch.rand(n), torch.randint(0, 2, (n,))
            m.update(x, t)
            xs.append(x), ts.append(t)
            allx, allt = torch.cat(xs)[-20:], torch.cat(ts)[-20:]
            torch.testing.assert_close(m.compute(), binary_auroc(allx, allt).double())

    def test_zero_scores_not_mistaken_for_empty(self) -> None:
        # real 0.0 scores at the tail of a full window must still be counted
        m = WindowedBinaryAUROC(max_num_samples=4)
        m.update(torch.tensor([0.9, 0.8, 0.0, 0.0]), torch.tensor([1, 0, 1, 0]))
        torch.testing.assert_close(m.compute(), binary_auroc(torch.tensor([0.9, 0.8, 0.0, 0.0]), torch.tensor([1, 0, 1, 0])).double())

    def test_class_suite(self) -> None:
        torch.manual_seed(9)
        input, target = torch.rand(8, 10), torch.randint(0, 2, (8, 10))
        self.run_class_implementation_tests(
            metric=WindowedBinaryAUROC(max_num_samples=30),
            state_names={"max_num_samples", "total_samples", "inputs", "targets", "weights"},
            update_kwargs={"input": input, "target": target},
            compute_result=binary_auroc(input[-3:].flatten(), target[-3:].flatten()).double(),
            # each of 4 ranks keeps its 20 samples; merged window holds all 80
            merge_and_compute_result=binary_auroc(input.flatten(), target.flatten()).double(),
            num_total_updates=8,
            num_processes=4,
        )
