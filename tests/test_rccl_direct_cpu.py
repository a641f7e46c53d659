"""Direct RCCL communicator plumbing that needs no GPU (parallel/rccl_direct.py): the entry
points resolve from torch's librccl, the unique id is 128 bytes, the env switch and the
non-CUDA guard keep every other path on torch.distributed."""

import pytest
import torch

from torcheval_amd.ops import native, native_loaded
from torcheval_amd.parallel import rccl_direct

pytestmark = pytest.mark.skipif(not native_loaded(), reason="native extension not built")


def test_entry_points_resolve():
    assert native().rccl_available()


def test_unique_id_is_128_bytes_and_fresh():
    a = torch.zeros(128, dtype=torch.uint8)
    b = torch.zeros(128, dtype=torch.uint8)
    native().rccl_unique_id(a)
    native().rccl_unique_id(b)
    assert a.any() and not torch.equal(a, b)
    with pytest.raises(RuntimeError):
        native().rccl_unique_id(torch.zeros(64, dtype=torch.uint8))


def test_env_switch(monkeypatch):
    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "0")
    assert not rccl_direct.enabled()
    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "1")
    assert rccl_direct.enabled()


def test_cpu_tensors_never_get_a_communicator():
    assert rccl_direct.comm_for(None, 2, torch.device("cpu")) is None


def test_dispatcher_schemas_declare_mutation():
    ag = str(torch.ops.torcheval_amd.rccl_all_gather.default._schema)
    ar = str(torch.ops.torcheval_amd.rccl_all_reduce.default._schema)
    assert "Tensor(a!) dst" in ag and "Tensor(a!) t" in ar and "Tensor(b!)? out" in ar


def _plan_metrics():
    from torcheval_amd.metrics import (
        BinaryBinnedAUPRC, BinaryNormalizedEntropy, BLEUScore, ClickThroughRate, Max, Mean, Min,
        MulticlassAccuracy, MulticlassBinnedPrecisionRecallCurve, MulticlassConfusionMatrix, MulticlassF1Score,
        MulticlassPrecision, MulticlassRecall, Perplexity, Sum, WeightedCalibration, WordErrorRate)
    from torcheval_amd.metrics.image.fid import FrechetInceptionDistance
    from torcheval_amd.metrics.metric import Metric

    class Mixed(Metric[torch.Tensor]):
        def __init__(self):
            super().__init__()
            self._add_state("f", torch.zeros(5, dtype=torch.float64), merge="sum")
            self._add_state("i", torch.zeros(3, dtype=torch.int64), merge="max")
            self._add_state("b", torch.zeros(7, dtype=torch.bool), merge="sum")
            self._add_state("h", torch.zeros(2, 9, dtype=torch.bfloat16), merge="min")
            self._add_state("big", torch.zeros(200, 200), merge="sum")

        def update(self, x):
            return self

        def compute(self):
            return self.f

        def merge_state(self, metrics):
            return self

    g = torch.Generator().manual_seed(0)
    x, y = torch.randn(64, 10, generator=g), torch.randint(0, 10, (64,), generator=g)
    out = [
        MulticlassAccuracy().update(x, y),
        MulticlassAccuracy(num_classes=10, average="macro").update(x, y),
        MulticlassPrecision(num_classes=10, average=None).update(x, y),
        MulticlassRecall(num_classes=10, average="macro").update(x, y),
        MulticlassF1Score(num_classes=10, average="weighted").update(x, y),
        MulticlassConfusionMatrix(300).update(torch.randn(64, 300, generator=g), torch.randint(0, 300, (64,), generator=g)),
        BinaryBinnedAUPRC(threshold=50).update(torch.rand(64, generator=g), y % 2),
        MulticlassBinnedPrecisionRecallCurve(num_classes=10, threshold=20).update(x.softmax(1), y),
        Mean().update(torch.randn(9, generator=g)), Sum().update(torch.randn(9, generator=g)),
        Max().update(torch.randn(9, generator=g)), Min().update(torch.randn(9, generator=g)),
        BinaryNormalizedEntropy().update(torch.rand(64, generator=g), (y % 2).float()),
        ClickThroughRate().update((y % 2).float()), WeightedCalibration().update(torch.rand(64, generator=g), (y % 2).float()),
        BLEUScore(n_gram=4).update(["the cat sat on the mat"], [["the cat sat on a mat"]]),
        Perplexity().update(torch.randn(2, 8, 10, generator=g), torch.randint(0, 10, (2, 8), generator=g)),
        WordErrorRate().update(["a b c"], ["a c c"]),
        Mixed(),
    ]
    fid = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=64)
    fid.update_activations(torch.randn(100, 64, generator=g), True)
    out.append(fid)
    return out


def test_direct_plan_specs_cover_the_buffer_and_views_match():
    """The direct-RCCL plan of every state-buffer layout (built here without a GPU): the
    all-reduce operands tile the groups and the error flag exactly once, and the native views of
    a result buffer (rccl_plan_views, what rccl_plan_sync returns) equal the layout's own views
    - dtype, shape and bytes - for every state."""
    from torcheval_amd.parallel import state_buffer as sbm

    checked = 0
    for m in _plan_metrics():
        sb = sbm.buffer_of(m)
        if sb is None:  # not a state-buffer layout (e.g. a variable-size error record)
            continue
        ops, assign = sbm.direct_plan_spec(sb, type(m))
        covered = torch.zeros(sb.buf.numel(), dtype=torch.int32)
        for kind, so, do, count, code, op in ops:
            assert kind == 0 and so == do
            es = torch.empty((), dtype={v: k for k, v in sbm._DT_CODE.items()}[code]).element_size()
            covered[so : so + count * es] += 1
        want = torch.zeros_like(covered)
        for gr in sb.groups:
            want[gr.off : gr.off + gr.nbytes] = 1
        if sb.flag_words:
            want[sb.flag_off : sb.flag_off + 4 * sb.flag_words] = 1
        assert torch.equal(covered, want), type(m).__name__
        plan = rccl_direct.plan_create(ops)
        rccl_direct.plan_set_views(plan, sbm.view_specs(assign))
        buf = torch.randint(0, 256, (sb.buf.numel(),), dtype=torch.uint8)
        got = native().rccl_plan_views(plan, buf)
        assert got[0].data_ptr() == buf.data_ptr() and len(got) == len(assign) + 1
        ref = sb.views(buf)
        if sb.flag_words:
            ref["_err"] = sb.flag_view(buf)
        for (name, dt, eo, n, shape, prop), v in zip(assign, got[1:]):
            r = ref[name]
            assert v.dtype == r.dtype and v.shape == r.shape, (type(m).__name__, name)
            assert v.data_ptr() == r.data_ptr(), (type(m).__name__, name)
            assert torch.equal(v.reshape(-1).view(torch.uint8), r.reshape(-1).view(torch.uint8)), name
            live = getattr(m, name)
            if live is None:  # an error flag not created yet: the synced copy gets the merged slot
                assert name == "_err"
                continue
            assert v.shape == live.shape and v.dtype == live.dtype, (type(m).__name__, name)
        checked += 1
    assert checked >= 15, checked


def test_int16_layouts_keep_the_gather_path():
    from torcheval_amd.metrics.metric import Metric
    from torcheval_amd.parallel import state_buffer as sbm

    class Short(Metric[torch.Tensor]):
        def __init__(self):
            super().__init__()
            self._add_state("s", torch.zeros(4, dtype=torch.int16), merge="sum")

        def update(self, x):
            return self

        def compute(self):
            return self.s

        def merge_state(self, metrics):
            return self

    assert sbm.direct_plan_spec(sbm.buffer_of(Short()), Short) is None


class _FakeRccl:
    """Stands in for the native all-reduce / all-gather of a ws-rank group as seen from one rank."""

    def __init__(self, ws, others, shift=0):
        self.ws, self.others, self.shift = ws, others, shift

    def rccl_all_reduce(self, handle, send, op, out):
        out.copy_(send + self.others)

    def rccl_all_gather(self, handle, src, dst):
        dst.copy_(torch.roll(torch.arange(1, self.ws + 1, dtype=torch.int32), self.shift))


@pytest.mark.parametrize("ws,rank", [(2, 0), (4, 3), (8, 5)])
def test_direct_comm_bootstrap_self_check(monkeypatch, ws, rank):
    import torcheval_amd.ops as ops
    from torcheval_amd.parallel import rccl_direct

    # what the other ranks contribute: sum over r != rank of [r + 1, ws - r]
    others = torch.tensor([sum(r + 1 for r in range(ws) if r != rank), sum(ws - r for r in range(ws) if r != rank)],
                          dtype=torch.int32)
    monkeypatch.setattr(ops, "native", lambda: _FakeRccl(ws, others))
    assert rccl_direct._self_check(1, ws, rank, torch.device("cpu"))
    monkeypatch.setattr(ops, "native", lambda: _FakeRccl(ws, others, shift=1))  # rank order mismatch
    with pytest.warns(UserWarning, match="bootstrap check"):
        assert not rccl_direct._self_check(1, ws, rank, torch.device("cpu"))
    monkeypatch.setattr(ops, "native", lambda: _FakeRccl(ws, others + 1))  # wrong reduction
    with pytest.warns(UserWarning, match="bootstrap check"):
        assert not rccl_direct._self_check(1, ws, rank, torch.device("cpu"))
