"""Contiguous per-metric state buffer: layout, in-place reset, rebuild on
rebinding, pickling, and eligibility."""

import copy
import pickle

import torch

from torcheval_amd.metrics import (
    BinaryAUROC,
    Mean,
    MeanSquaredError,
    Metric,
    MulticlassAccuracy,
    MulticlassConfusionMatrix,
    Sum,
)
from torcheval_amd.parallel.state_buffer import SMALL_STATE_BYTES, buffer_of, plan_summary


def _storage(t: torch.Tensor) -> int:
    return t.untyped_storage().data_ptr()


def test_states_become_views_of_one_buffer():
    m = MulticlassAccuracy(num_classes=4, average="macro")
    m.update(torch.eye(4), torch.arange(4))
    before = m.compute().clone()
    sb = buffer_of(m)
    assert sb is not None
    assert _storage(m.num_correct) == _storage(m.num_total) == sb.buf.data_ptr()
    torch.testing.assert_close(m.compute(), before)
    m.update(torch.eye(4), torch.tensor([0, 1, 2, 0]))  # in-place updates land in the buffer
    assert buffer_of(m, build=False) is sb
    assert float(sb.views(sb.buf)["num_correct"].sum()) == 7.0


def test_reset_is_one_copy_and_keeps_views():
    m = Sum()
    m.update(torch.tensor([1.0, 2.0]))
    sb = buffer_of(m)
    ptr = m.weighted_sum.data_ptr()
    m.reset()
    assert m.weighted_sum.data_ptr() == ptr and float(m.weighted_sum) == 0.0
    assert buffer_of(m, build=False) is sb
    m.update(torch.tensor([3.0]))
    assert float(m.compute()) == 3.0


def test_compute_then_reset_keeps_the_returned_value():
    """``v = m.compute(); m.reset()`` must leave ``v`` alone even though the reset
    restores the state buffer in place (reference metric.py:120-147 rebinds instead)."""
    from torcheval_amd.metrics import Max, Min

    s = Sum().update(torch.tensor([1.0, 2.0]))
    mx = Max().update(torch.tensor([1.0, 5.0]))
    mn = Min().update(torch.tensor([1.0, -5.0]))
    cm = MulticlassConfusionMatrix(3).update(torch.eye(3), torch.arange(3))
    for m in (s, mx, mn, cm):
        assert buffer_of(m) is not None  # what the first sync builds
    got = [m.compute() for m in (s, mx, mn, cm)] + [cm.normalized(None)]
    for m in (s, mx, mn, cm):
        m.reset()
    assert float(got[0]) == 3.0 and float(got[1]) == 5.0 and float(got[2]) == -5.0
    assert torch.equal(got[3], torch.eye(3)) and torch.equal(got[4], torch.eye(3))
    assert float(cm.compute().sum()) == 0.0


def test_rebinding_rebuilds_the_buffer():
    m = Mean()
    m.update(torch.tensor([1.0, 3.0]))
    sb = buffer_of(m)
    m.load_state_dict({"weighted_sum": torch.tensor(10.0, dtype=torch.float64),
                       "weights": torch.tensor(4.0, dtype=torch.float64)})
    assert buffer_of(m, build=False) is None  # the views were replaced
    sb2 = buffer_of(m)
    assert sb2 is not sb
    assert float(m.compute()) == 2.5


def test_pickle_and_deepcopy_rebuild():
    m = MulticlassAccuracy()
    m.update(torch.randn(16, 5), torch.randint(0, 5, (16,)))
    buffer_of(m)
    for clone in (pickle.loads(pickle.dumps(m)), copy.deepcopy(m)):
        torch.testing.assert_close(clone.compute(), m.compute())
        assert buffer_of(clone, build=False) is None
        assert buffer_of(clone) is not None
        clone.update(torch.randn(4, 5), torch.randint(0, 5, (4,)))
        assert float(clone.num_total) == 20.0 and float(m.num_total) == 16.0


def test_layout_groups_and_collectives():
    small = plan_summary(MulticlassAccuracy())
    assert small["collectives"] == 1 and not small["reduce_groups"] and small["flag_words"] == 0
    assert plan_summary(MulticlassAccuracy(num_classes=3, average="macro"))["flag_words"] == 1
    big = plan_summary(MulticlassConfusionMatrix(1000))
    assert big["reduce_groups"][0][3] == 1000 * 1000 * 4 > SMALL_STATE_BYTES
    assert big["flag_words"] == 3 and big["collectives"] == 2


class _Lazy(Metric[torch.Tensor]):
    """A sum state promoted from () to [k] by its first update (like MSE's lazy shapes)."""

    def __init__(self) -> None:
        super().__init__()
        self._add_state("s", torch.tensor(0.0), merge="sum")

    def update(self, x):
        if self.s.ndim == 0:
            self.s = torch.zeros(x.shape[1])
        self.s += x.sum(0)
        return self

    def compute(self):
        return self.s

    def merge_state(self, metrics):
        for m in metrics:
            self.s = self.s + m.s
        return self


def test_ineligible_and_lazily_shaped_metrics():
    assert buffer_of(BinaryAUROC()) is None  # cat states: all-gather-v engine
    assert buffer_of(MeanSquaredError()) is None  # untyped (custom merge) states
    m = _Lazy().update(torch.ones(2, 3))
    sb = buffer_of(m)
    assert sb is not None and sb.default_img is None
    m.reset()  # generic path restores the scalar default
    assert m.s.shape == torch.Size([])
    assert buffer_of(m, build=False) is None
    m.update(torch.ones(4, 2))
    assert m.compute().tolist() == [4.0, 4.0]


def test_sorted_run_merge_without_native(monkeypatch):
    """the synced-AUROC merge path must not need _C (or launch K3m) when the
    native path is off; a stable sort of the concatenated runs is the same merge."""
    from torcheval_amd.metrics.functional import binary_auprc, binary_auroc
    from torcheval_amd.metrics.functional.classification import _curve

    g = torch.Generator().manual_seed(4)
    runs = [torch.sort(torch.randint(0, 30, (n,), generator=g).float() / 30, descending=True)[0]
            for n in (50, 1, 77)]
    ts = [torch.randint(0, 2, (r.numel(),), generator=g) for r in runs]
    want = (binary_auroc(torch.cat(runs), torch.cat(ts)), binary_auprc(torch.cat(runs), torch.cat(ts)))
    for loaded in (True, False):
        monkeypatch.setattr(_curve, "native_loaded", lambda: loaded)
        roc, pr = _curve.merged_areas(runs, ts, None, roc=True, pr=True)
        torch.testing.assert_close(roc[0], want[0].double(), rtol=1e-12, atol=1e-12)
        torch.testing.assert_close(pr[0], want[1].double(), rtol=1e-6, atol=1e-6)
