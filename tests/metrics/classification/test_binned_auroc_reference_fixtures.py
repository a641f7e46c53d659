"""The reference's own multiclass binned AUROC fixtures, pinned.

Reference: tests/metrics/functional/classification/test_binned_auroc.py:178-234 (functional,
macro 0.4000 and a per-SAMPLE 5-vector) and tests/metrics/classification/test_binned_auroc.py:
144-209 (class, seeded 0.5013020634651184; 0.625 and [0.25, 0.25, 1.0, 1.0] over 2 processes).
``one_vs_rest=True`` is the opt-in per-class form.  The ``gpu`` variants feed cuda:0 tensors.
"""

import pytest
import torch

from torcheval_amd.metrics import MulticlassBinnedAUROC
from torcheval_amd.metrics.functional import multiclass_auroc, multiclass_binned_auroc
from torcheval_amd.utils.test_utils.metric_class_tester import MetricClassTester

THR5 = torch.tensor([0.0, 0.25, 0.5, 0.75, 1.0])
X = torch.tensor([[0.1, 0.2, 0.1], [0.4, 0.2, 0.1], [0.6, 0.1, 0.2], [0.4, 0.2, 0.3], [0.6, 0.2, 0.4]])
Y = torch.tensor([0, 1, 2, 1, 0])


def _devices():
    return ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("dev", _devices())
def test_functional_fixture(dev):
    auroc, thr = multiclass_binned_auroc(X.to(dev), Y.to(dev), num_classes=3, threshold=5)
    torch.testing.assert_close(auroc.cpu(), torch.tensor(0.4000), atol=1e-8, rtol=1e-5)
    torch.testing.assert_close(thr.cpu(), THR5)
    auroc, _ = multiclass_binned_auroc(X.to(dev), Y.to(dev), num_classes=3, threshold=5, average=None)
    torch.testing.assert_close(auroc.cpu(), torch.tensor([0.5, 0.25, 0.25, 0.0, 1.0]), atol=1e-8, rtol=1e-5)
    assert auroc.dtype == torch.float32


@pytest.mark.parametrize("dev", _devices())
def test_one_vs_rest_opt_in(dev):
    per_class, _ = multiclass_binned_auroc(X.to(dev), Y.to(dev), num_classes=3, threshold=5, average=None,
                                           one_vs_rest=True)
    assert per_class.shape == (3,)
    # thresholds covering every distinct score: the binned one-vs-rest curve is the exact one
    thr = torch.cat([torch.tensor([0.0]), X.unique(), torch.tensor([1.0])]).unique()
    fine, _ = multiclass_binned_auroc(X.to(dev), Y.to(dev), num_classes=3, threshold=thr.to(dev), average=None,
                                      one_vs_rest=True)
    torch.testing.assert_close(fine.cpu().double(), multiclass_auroc(X, Y, num_classes=3, average=None).double(),
                               atol=1e-6, rtol=1e-6)
    m = MulticlassBinnedAUROC(num_classes=3, threshold=5, average=None, one_vs_rest=True, device=dev)
    m.update(X.to(dev), Y.to(dev))
    torch.testing.assert_close(m.compute()[0], per_class)


class TestMulticlassBinnedAUROCFixtures(MetricClassTester):
    def test_class_base(self) -> None:
        torch.manual_seed(123)
        inp = 10 * torch.rand(8, 16, 4)
        inp = inp.abs() / inp.abs().sum(dim=-1, keepdim=True)
        tgt = torch.randint(high=4, size=(8, 16))
        self.run_class_implementation_tests(
            metric=MulticlassBinnedAUROC(num_classes=4, threshold=5),
            state_names={"inputs", "targets"},
            update_kwargs={"input": inp, "target": tgt},
            compute_result=(torch.tensor(0.5013020634651184), THR5),
        )

    def test_class_average_options(self) -> None:
        inp = torch.tensor([[[0.16, 0.04, 0.8]], [[0.1, 0.7, 0.2]], [[0.16, 0.8, 0.04]], [[0.16, 0.04, 0.8]]])
        tgt = torch.tensor([[0], [0], [1], [2]])
        for avg, want in (("macro", torch.tensor(0.625)), (None, torch.tensor([0.25, 0.25, 1.0, 1.0]))):
            self.run_class_implementation_tests(
                metric=MulticlassBinnedAUROC(num_classes=3, threshold=5, average=avg),
                state_names={"inputs", "targets"},
                update_kwargs={"input": inp, "target": tgt},
                num_total_updates=4,
                num_processes=2,
                compute_result=(want, THR5),
            )
