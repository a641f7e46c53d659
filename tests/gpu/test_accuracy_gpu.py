"""MulticlassAccuracy on MI355X: HIP path vs the CPU/ATen path on identical data."""

import pytest
import torch

from torcheval_amd.metrics import BinaryAccuracy, MulticlassAccuracy
from torcheval_amd.metrics.functional import binary_accuracy, multiclass_accuracy
from torcheval_amd.metrics.toolkit import get_synced_metric

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("average,k", [("micro", 1), ("micro", 3), ("macro", 1), (None, 1), ("macro", 2)])
def test_class_gpu_matches_cpu(average, k):
    torch.manual_seed(0)
    C = 37
    kwargs = dict(average=average, k=k, num_classes=None if average == "micro" else C)
    m_cpu = MulticlassAccuracy(**kwargs)
    m_gpu = MulticlassAccuracy(**kwargs, device=torch.device("cuda"))
    for _ in range(5):
        x = torch.randn(1000, C)
        y = torch.randint(0, C, (1000,))
        m_cpu.update(x, y)
        m_gpu.update(x.cuda(), y.cuda())
    torch.testing.assert_close(m_gpu.compute().cpu(), m_cpu.compute())
    x = torch.randn(513, C)
    y = torch.randint(0, C, (513,))
    torch.testing.assert_close(
        multiclass_accuracy(x.cuda(), y.cuda(), **kwargs).cpu(), multiclass_accuracy(x, y, **kwargs)
    )


def test_out_of_range_target_raises_at_compute():
    m = MulticlassAccuracy(average="macro", num_classes=4, device=torch.device("cuda"))
    m.update(torch.randn(8, 4).cuda(), torch.tensor([0, 1, 2, 3, 4, 0, 1, 2]).cuda())
    with pytest.raises(RuntimeError, match="out of bounds"):
        m.compute()


def test_binary_gpu():
    x = torch.rand(10000)
    y = torch.randint(0, 2, (10000,))
    m = BinaryAccuracy(threshold=0.7, device=torch.device("cuda"))
    m.update(x.cuda(), y.cuda())
    torch.testing.assert_close(m.compute().cpu(), binary_accuracy(x, y, threshold=0.7))


def test_ws1_sync_returns_same_object():
    m = MulticlassAccuracy(device=torch.device("cuda"))
    assert get_synced_metric(m) is m
