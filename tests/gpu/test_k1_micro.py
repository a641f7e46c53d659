"""K1 micro kernel (MulticlassAccuracy micro, k=1): adversarial rows against torch.argmax on
CPU, and the deferred fold of its pending per-wave counts (compute / sync / state_dict / copy /
reset / HIP-graph replay all see exactly the reference counts)."""

import copy
import pickle

import pytest
import torch

from torcheval_amd.metrics import MulticlassAccuracy
from torcheval_amd.utils.graphs import GraphedUpdate

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ref_argmax(x: torch.Tensor) -> torch.Tensor:
    return x.float().argmax(1)  # CPU torch.argmax: NaN is the max, first index wins


def _adversarial(n, c, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, c, generator=g)
    y = torch.randint(0, c, (n,), generator=g)
    hit = torch.rand(n, generator=g) < 0.6
    x[hit, y[hit]] = 10.0
    r = torch.arange(n)
    tb = (r % 7 == 0) & (y > 0)
    x[tb, 0] = x[tb, y[tb]]  # an earlier column ties the target's max: wrong
    ta = r % 11 == 0
    x[ta, c - 1] = x[ta, y[ta]]  # a later tie: still right
    x[r % 13 == 0, c // 2] = float("nan")
    x[r % 17 == 0, 1] = float("inf")
    z = r % 19 == 0
    x[z] = 0.0
    x[z, 0] = -0.0
    y[r % 23 == 0] = c + 5  # out-of-range targets never count as correct (micro: no error)
    y[r % 29 == 0] = -1
    return x.to(dtype), y


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("c", [33, 257, 1000, 1024, 2048])
@pytest.mark.parametrize("tdtype", [torch.int64, torch.int32])
def test_micro_kernel_matches_argmax(dtype, c, tdtype):
    if dtype == torch.float32 and c > 1024:
        pytest.skip("f32 rows over 1024 columns take the general kernel")
    x, y = _adversarial(4000, c, dtype, c)
    want = ((_ref_argmax(x) == y).sum().item(), y.numel())
    m = MulticlassAccuracy(device=DEV)
    xd, yd = x.to(DEV), y.to(tdtype).to(DEV)
    for _ in range(3):
        m.update(xd, yd)
    assert m.__dict__["_pend_dirty"]  # the micro kernel ran in deferred-fold mode
    assert float(m.num_correct) == 3 * want[0] and float(m.num_total) == 3 * want[1]
    assert not m.__dict__["_pend_dirty"]


def test_deferred_fold_semantics():
    x, y = _adversarial(8192, 1000, torch.float32, 1)
    xd, yd = x.to(DEV), y.to(DEV)
    hits = (_ref_argmax(x) == y).sum().item()
    m = MulticlassAccuracy(device=DEV)
    m.update(xd, yd).update(xd, yd)
    torch.testing.assert_close(m.compute().cpu(), torch.tensor(hits / 8192))  # fold + divide
    m.update(xd, yd)
    assert m.state_dict()["num_correct"].item() == 3 * hits  # state reads fold
    m.update(xd, yd)
    for clone in (copy.deepcopy(m), pickle.loads(pickle.dumps(m)), copy.copy(m)):
        assert float(clone.num_correct) == 4 * hits
    assert float(m.num_correct) == 4 * hits
    m.update(xd, yd)
    m.reset()  # pending counts are discarded with the rest of the state
    assert float(m.num_correct) == 0.0 and float(m.num_total) == 0.0
    m.update(xd, yd)
    m.load_state_dict({"num_correct": torch.tensor(5.0, device=DEV), "num_total": torch.tensor(10.0, device=DEV)})
    assert float(m.num_correct) == 5.0  # the replaced value's pending counts do not leak in
    m.update(xd, yd)
    assert float(m.num_correct) == 5.0 + hits


def test_graph_replays_are_folded():
    x, y = _adversarial(8192, 1000, torch.float32, 2)
    xd, yd = x.to(DEV), y.to(DEV)
    hits = (_ref_argmax(x) == y).sum().item()
    m = MulticlassAccuracy(device=DEV)
    step = GraphedUpdate(m, xd, yd)
    for _ in range(5):
        step(xd, yd)
    assert float(m.num_correct) == 5 * hits and float(m.num_total) == 5 * 8192


@pytest.mark.parametrize("n", [1, 7, 9, 8191, 8193, 20001])
def test_micro_kernel_ragged_and_grid_stride_rows(n):
    """8-wave workgroups, one wave per row: a partial last workgroup (n % 8 != 0) and more rows
    than the 1024 x 8 waves of one grid pass (grid-stride)."""
    x, y = _adversarial(n, 1000, torch.float32, 3)
    want = (_ref_argmax(x) == y).sum().item()
    m = MulticlassAccuracy(device=DEV)
    m.update(x.to(DEV), y.to(DEV))
    assert float(m.num_correct) == want and float(m.num_total) == n
