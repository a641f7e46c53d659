"""AUC(reorder=True) on ROCm: K3a ascending stable sort with y as payload + K3t trapezoids,
against the ATen form (torch.sort(stable) + gather + trapz; reference
torcheval/metrics/functional/aggregation/auc.py:10-33) on the CPU."""

import pytest
import torch

from torcheval_amd.metrics import AUC
from torcheval_amd.metrics.functional import auc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(x, y):
    x2 = x if x.ndim == 2 else x.unsqueeze(0)
    y2 = y if y.ndim == 2 else y.unsqueeze(0)
    xs, idx = torch.sort(x2.double(), dim=1, stable=True)
    return torch.trapz(y2.double().gather(1, idx), xs)


def test_reference_docstring_fixtures():
    y = torch.tensor([[0, 4, 0, 4, 3], [1, 1, 2, 1, 1], [4, 3, 1, 4, 4], [1, 0, 0, 3, 0]])
    x = torch.tensor([[0.2535, 0.1138, 0.1324, 0.1887, 0.3117],
                      [0.1434, 0.4404, 0.1100, 0.1178, 0.1883],
                      [0.2344, 0.1743, 0.3110, 0.0393, 0.2410],
                      [0.1381, 0.1564, 0.0320, 0.2220, 0.4515]])
    got = auc(x.to(DEV), y.to(DEV), reorder=True).cpu()
    torch.testing.assert_close(got, torch.tensor([0.3667, 0.3343, 0.8843, 0.5048]), rtol=0, atol=1e-4)
    m = AUC(device=DEV)
    m.update(torch.tensor([0, .1, .13, .2], device=DEV), torch.tensor([1, 1, 2, 4], device=DEV))
    m.update(torch.tensor([1., 2., .1, 3.], device=DEV), torch.tensor([1, 2, 3, 2], device=DEV))
    torch.testing.assert_close(m.compute().cpu(), torch.tensor([5.8850]), rtol=0, atol=1e-4)
    m = AUC(n_tasks=2, device=DEV)
    m.update(torch.tensor([[0.3941, 0.2980, 0.3080], [0.1448, 0.6090, 0.2462]], device=DEV),
             torch.tensor([[1, 0, 4], [0, 4, 2]], device=DEV))
    m.update(torch.tensor([[0.4562, 0.1200, 0.4238], [0.4076, 0.4448, 0.1476]], device=DEV),
             torch.tensor([[3, 4, 3], [2, 0, 4]], device=DEV))
    torch.testing.assert_close(m.compute().cpu(), torch.tensor([0.7479, 0.9898]), rtol=0, atol=1e-4)


@pytest.mark.parametrize("tasks,n", [(1, 2), (1, 1000), (3, 4097), (4, 1_000_000), (9, 20_000)])
def test_matches_aten(tasks, n):
    g = torch.Generator().manual_seed(n + tasks)
    x = torch.rand(tasks, n, generator=g)
    y = torch.randn(tasks, n, generator=g)
    got = auc(x.to(DEV), y.to(DEV), reorder=True).cpu()
    ref = _ref(x, y).float()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * float(y.abs().max()))


def test_ties_keep_input_order():
    # many equal x: the y order inside a tie group decides the boundary trapezoids (stable sort)
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 50, (3, 100_000), generator=g).float() / 7
    x[:, ::5] = -0.0  # -0.0 and 0.0 tie, as in torch.sort
    x[:, 1::7] = 0.0
    y = torch.randn(3, 100_000, generator=g)
    got = auc(x.to(DEV), y.to(DEV), reorder=True).cpu()
    ref = _ref(x, y).float()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-4)


def test_single_point_nan_and_no_reorder():
    one = auc(torch.tensor([0.5], device=DEV), torch.tensor([2.0], device=DEV), reorder=True).cpu()
    assert one.tolist() == [0.0]
    x = torch.rand(2, 100)
    x[1, 7] = float("nan")
    y = torch.rand(2, 100)
    got = auc(x.to(DEV), y.to(DEV), reorder=True).cpu()
    assert torch.isnan(got[1]) and not torch.isnan(got[0])
    torch.testing.assert_close(got[0], _ref(x[:1], y[:1]).float()[0], rtol=1e-5, atol=1e-6)
    # reorder=False keeps the ATen trapz over the given order
    torch.testing.assert_close(auc(x.to(DEV), y.to(DEV)).cpu(), torch.trapz(y, x), equal_nan=True)
