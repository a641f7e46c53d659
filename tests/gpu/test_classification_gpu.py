"""Class metrics on MI355X vs the CPU path on identical data (HIP kernels vs ATen)."""

import pytest
import torch

import torcheval_amd.metrics as M

pytestmark = pytest.mark.gpu


def _run(metric_fn, batches, **kw):
    cpu = metric_fn(**kw)
    gpu = metric_fn(**kw, device=torch.device("cuda"))
    for b in batches:
        cpu.update(*b)
        gpu.update(*[t.cuda() for t in b])
    return cpu.compute(), gpu.compute()


def _close(a, b):
    if isinstance(a, (tuple, list)):
        for x, y in zip(a, b):
            _close(x, y)
    else:
        torch.testing.assert_close(b.cpu(), a, rtol=1e-5, atol=1e-6, equal_nan=True)


@pytest.mark.parametrize("cls,kw", [
    (M.MulticlassPrecision, dict(num_classes=7, average="macro")),
    (M.MulticlassPrecision, dict(num_classes=7, average=None)),
    (M.MulticlassPrecision, dict()),
    (M.MulticlassRecall, dict(num_classes=7, average="weighted")),
    (M.MulticlassRecall, dict()),
    (M.MulticlassF1Score, dict(num_classes=7, average="macro")),
    (M.MulticlassF1Score, dict()),
    (M.MulticlassConfusionMatrix, dict(num_classes=7)),
    (M.MulticlassAUROC, dict(num_classes=7)),
    (M.MulticlassAUPRC, dict(num_classes=7)),
    (M.MulticlassBinnedAUPRC, dict(num_classes=7, threshold=20)),
    (M.MulticlassBinnedPrecisionRecallCurve, dict(num_classes=7, threshold=20)),
])
def test_multiclass_metrics(cls, kw):
    g = torch.Generator().manual_seed(1)
    batches = [(torch.rand(300, 7, generator=g), torch.randint(0, 7, (300,), generator=g)) for _ in range(4)]
    _close(*_run(cls, batches, **kw))


@pytest.mark.parametrize("cls,kw", [
    (M.BinaryPrecision, dict(threshold=0.4)),
    (M.BinaryRecall, dict()),
    (M.BinaryF1Score, dict()),
    (M.BinaryConfusionMatrix, dict()),
    (M.BinaryAUROC, dict()),
    (M.BinaryAUPRC, dict()),
    (M.BinaryBinnedAUROC, dict(threshold=30)),
    (M.BinaryBinnedAUPRC, dict(threshold=30)),
    (M.BinaryBinnedPrecisionRecallCurve, dict(threshold=30)),
    (M.BinaryNormalizedEntropy, dict()),
])
def test_binary_metrics(cls, kw):
    g = torch.Generator().manual_seed(2)
    batches = []
    for _ in range(4):
        x = torch.rand(500, generator=g)
        t = torch.randint(0, 2, (500,), generator=g)
        batches.append((x, t.float() if cls is M.BinaryNormalizedEntropy else t))
    _close(*_run(cls, batches, **kw))


def test_multilabel_binned_and_auprc():
    g = torch.Generator().manual_seed(3)
    batches = [(torch.rand(200, 5, generator=g), torch.randint(0, 2, (200, 5), generator=g)) for _ in range(3)]
    _close(*_run(M.MultilabelAUPRC, batches, num_labels=5))
    _close(*_run(M.MultilabelBinnedAUPRC, batches, num_labels=5, threshold=15))
    _close(*_run(M.MultilabelBinnedPrecisionRecallCurve, batches, num_labels=5, threshold=15))
