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


def test_fast_path_keeps_the_reference_shape_check():
    """MulticlassAccuracy(num_classes=10) on [N, 1000] scores: the K1 fast path declines and
    the reference's ValueError is raised (reference accuracy.py:340-346)."""
    dev = torch.device("cuda")
    m = MulticlassAccuracy(num_classes=10, device=dev)
    assert m._fast
    with pytest.raises(ValueError, match="input should have shape of"):
        m.update(torch.randn(64, 1000, device=dev), torch.randint(0, 10, (64,), device=dev))
    m.update(torch.randn(64, 10, device=dev), torch.randint(0, 10, (64,), device=dev))  # matching: fast path
    assert float(m.num_total) == 64.0


def test_state_buffer_sync_on_rccl_one_rank():
    """The contiguous state buffer under a 1-rank RCCL group (collectives forced): same
    results as local compute, inputs untouched, and a reset keeps the kernel's pointers."""
    import socket

    import torch.distributed as dist

    from torcheval_amd.metrics import MulticlassConfusionMatrix
    from torcheval_amd.metrics.toolkit import get_synced_metric, sync_and_compute
    from torcheval_amd.parallel.collectives import collectives_at_world_size_1
    from torcheval_amd.parallel.state_buffer import buffer_of

    dev = torch.device("cuda", 0)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        x = torch.randn(4096, 1000, device=dev)
        y = torch.randint(0, 1000, (4096,), device=dev)
        acc = MulticlassAccuracy(device=dev).update(x, y)
        cm = MulticlassConfusionMatrix(1000, device=dev).update(x, y)
        with collectives_at_world_size_1():
            for m in (acc, cm):
                local = m.compute().clone()
                torch.testing.assert_close(sync_and_compute(m), local)
                torch.testing.assert_close(m.compute(), local)  # inputs untouched
        # the confusion matrix's flag rides its all-reduce (one collective): a bad label on
        # this rank still raises from the synced copy, whose states match local compute
        from torcheval_amd.parallel.state_buffer import _plan_for

        cm_sb = buffer_of(cm, build=False)
        assert _plan_for(cm_sb, dist.group.WORLD, 1, cm).fused
        bad = y.clone()
        bad[7] = 1000 + 3
        cm2 = MulticlassConfusionMatrix(1000, device=dev).update(x, bad)
        with collectives_at_world_size_1():
            synced = get_synced_metric(cm2)
        assert synced._err.tolist()[0] != 0 and synced._err.tolist()[1] == 1003
        with pytest.raises(ValueError):
            synced.compute()
        sb = buffer_of(acc, build=False)
        assert sb is not None
        ptr = acc.num_correct.data_ptr()
        acc.reset()
        assert acc.num_correct.data_ptr() == ptr and float(acc.num_total) == 0.0
        acc.update(x, y)
        torch.testing.assert_close(acc.compute(), (x.argmax(1) == y).float().mean())
    finally:
        dist.destroy_process_group()


def test_binary_gpu():
    x = torch.rand(10000)
    y = torch.randint(0, 2, (10000,))
    m = BinaryAccuracy(threshold=0.7, device=torch.device("cuda"))
    m.update(x.cuda(), y.cuda())
    torch.testing.assert_close(m.compute().cpu(), binary_accuracy(x, y, threshold=0.7))


def test_ws1_sync_returns_same_object():
    m = MulticlassAccuracy(device=torch.device("cuda"))
    assert get_synced_metric(m) is m


# ----------------------------------------------------------------------------- K2 multilabel
_CRIT = ["exact_match", "hamming", "overlap", "contain", "belong"]


@pytest.mark.parametrize("criteria", _CRIT)
@pytest.mark.parametrize("shape", [(1, 1), (37, 5), (8192, 1000), (300, 1001)])
@pytest.mark.parametrize("tdtype", [torch.int64, torch.float32, torch.bool, torch.uint8, torch.int32])
def test_k2_multilabel_threshold(criteria, shape, tdtype):
    from torcheval_amd.metrics.functional import multilabel_accuracy

    g = torch.Generator().manual_seed(shape[0] * 31 + shape[1])
    x = torch.rand(shape, generator=g)
    x[0, 0] = float("nan")  # NaN >= threshold in the reference (where(x < thr, 0, 1))
    # sparse targets so overlap / contain / belong rows are a mix of true and false
    t = (torch.rand(shape, generator=g) < 0.3).to(tdtype)
    # bool targets: the reference's `input - target` rejects bool, so the oracle uses int labels
    ref = multilabel_accuracy(x, t.long(), criteria=criteria)
    got = multilabel_accuracy(x.cuda(), t.cuda(), criteria=criteria)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=1e-6)


@pytest.mark.parametrize("criteria", _CRIT)
@pytest.mark.parametrize("k", [2, 3, 5])
@pytest.mark.parametrize("c", [3, 64, 65, 1000, 2048])
def test_k2_topk_multilabel(criteria, k, c):
    from torcheval_amd.metrics.functional import topk_multilabel_accuracy

    if k > c:
        pytest.skip("k > c")
    g = torch.Generator().manual_seed(c * 7 + k)
    x = torch.rand(257, c, generator=g)
    t = (torch.rand(257, c, generator=g) < 0.05).long()
    # plant exact matches so exact / contain rows exist
    top = x[:50].topk(k, dim=-1).indices
    t[:50] = 0
    t[:50].scatter_(1, top, 1)
    ref = topk_multilabel_accuracy(x, t, criteria=criteria, k=k)
    got = topk_multilabel_accuracy(x.cuda(), t.cuda(), criteria=criteria, k=k)
    torch.testing.assert_close(got.cpu(), ref, rtol=0, atol=1e-6)


def test_k2_class_states_and_bf16():
    from torcheval_amd.metrics import MultilabelAccuracy, TopKMultilabelAccuracy
    from torcheval_amd.metrics.functional import multilabel_accuracy, topk_multilabel_accuracy

    g = torch.Generator().manual_seed(0)
    xs = [torch.rand(512, 100, generator=g) for _ in range(4)]
    ts = [(torch.rand(512, 100, generator=g) < 0.5).long() for _ in range(4)]
    for crit in _CRIT:
        m = MultilabelAccuracy(criteria=crit, device="cuda")
        mk = TopKMultilabelAccuracy(criteria=crit, k=3, device="cuda")
        for x, t in zip(xs, ts):
            m.update(x.cuda().bfloat16(), t.cuda())
            mk.update(x.cuda(), t.cuda())
        X, T = torch.cat(xs), torch.cat(ts)
        torch.testing.assert_close(m.compute().cpu(), multilabel_accuracy(X.bfloat16().float(), T, criteria=crit))
        torch.testing.assert_close(mk.compute().cpu(), topk_multilabel_accuracy(X, T, criteria=crit, k=3))


# ----------------------------------------------------------------------------- HIP graphs
def test_graphed_update_matches_eager():
    from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix, MultilabelAccuracy
    from torcheval_amd.utils.graphs import GraphedUpdate

    g = torch.Generator(device="cuda").manual_seed(0)
    xs = [torch.randn(64, 10, device="cuda", generator=g) for _ in range(20)]
    ys = [torch.randint(0, 10, (64,), device="cuda", generator=g) for _ in range(20)]
    for make in (lambda: MulticlassAccuracy(device="cuda"),
                 lambda: MulticlassAccuracy(average="macro", num_classes=10, device="cuda"),
                 lambda: MulticlassConfusionMatrix(10, device="cuda")):
        eager, graphed = make(), make()
        step = GraphedUpdate(graphed, xs[0], ys[0])
        for x, y in zip(xs, ys):
            eager.update(x, y)
            step(x, y)
        torch.testing.assert_close(graphed.compute(), eager.compute())
    ml_e, ml_g = MultilabelAccuracy(criteria="hamming", device="cuda"), MultilabelAccuracy(criteria="hamming", device="cuda")
    t = [(torch.rand(64, 10, device="cuda") < 0.5).long() for _ in range(5)]
    step = GraphedUpdate(ml_g, xs[0].sigmoid(), t[0])
    for x, tt in zip(xs, t):
        ml_e.update(x.sigmoid(), tt)
        step(x.sigmoid(), tt)
    torch.testing.assert_close(ml_g.compute(), ml_e.compute())


def test_graphed_update_rejects_rebinding_metric():
    from torcheval_amd.metrics import Metric, PeakSignalNoiseRatio
    from torcheval_amd.utils.graphs import GraphedUpdate

    class Rebinding(Metric):
        def __init__(self):
            super().__init__(device="cuda")
            self._add_state("total", torch.zeros((), device="cuda"))

        def update(self, x):
            self.total = self.total + x.sum()  # new tensor each call: not replayable
            return self

        def compute(self):
            return self.total

        def merge_state(self, metrics):
            return self

    with pytest.raises(RuntimeError, match="rebinds its states"):
        GraphedUpdate(Rebinding(), torch.rand(8, device="cuda"))
    class HostCopy(Rebinding):
        def update(self, x):
            self.total += torch.tensor(float(x.numel()), device="cuda")  # host -> device copy
            return self

    # an update that copies host data to the device cannot be recorded at all
    with pytest.raises(RuntimeError, match="cannot be captured"):
        GraphedUpdate(HostCopy(), torch.rand(8, device="cuda"))
    # PSNR's update is one K5b launch into its states: it records and replays like the eager path
    x, t = torch.rand(4, 3, 8, 8, device="cuda"), torch.rand(4, 3, 8, 8, device="cuda")
    graphed_m, eager_m = PeakSignalNoiseRatio(device="cuda"), PeakSignalNoiseRatio(device="cuda")
    step = GraphedUpdate(graphed_m, x, t)
    for _ in range(3):
        x.copy_(torch.rand_like(x))
        step(x, t)
        eager_m.update(x, t)
    torch.testing.assert_close(graphed_m.compute(), eager_m.compute())


@pytest.mark.gpu
def test_graphed_update_reports_its_measured_cost():
    """GraphedUpdate times direct updates against replays at construction and warns when the
    replay is slower (one-kernel updates on this runtime); the timing updates leave no trace."""
    import warnings

    from torcheval_amd.utils.graphs import GraphedUpdate

    x = torch.randn(8, 6, device="cuda")
    y = torch.randint(0, 6, (8,), device="cuda")
    m = MulticlassAccuracy(device="cuda")
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        step = GraphedUpdate(m, x, y)
    assert step.direct_us > 0 and step.replay_us > 0
    slower = [w for w in rec if "graph replay costs" in str(w.message)]
    assert bool(slower) == (step.replay_us > step.direct_us)
    assert float(m.compute().nan_to_num(-1)) == -1  # no samples counted by the timing runs
    step(x, y)
    ref = MulticlassAccuracy(device="cuda")
    ref.update(x, y)
    torch.testing.assert_close(m.compute(), ref.compute())
    print(f"GraphedUpdate bs=8: direct {step.direct_us:.1f} us, replay {step.replay_us:.1f} us")


@pytest.mark.gpu
def test_graphed_update_of_several_metrics():
    """One graph for the updates of five metrics fed the same batch: the states after N replays
    equal N direct updates of twins; the timing runs leave no trace; the measured costs print."""
    from torcheval_amd.metrics import (
        MulticlassConfusionMatrix,
        MulticlassF1Score,
        MulticlassPrecision,
        MulticlassRecall,
    )
    from torcheval_amd.utils.graphs import GraphedUpdate

    def five():
        return [
            MulticlassAccuracy(num_classes=6, device="cuda"),
            MulticlassPrecision(num_classes=6, average="macro", device="cuda"),
            MulticlassRecall(num_classes=6, device="cuda"),
            MulticlassF1Score(num_classes=6, average=None, device="cuda"),
            MulticlassConfusionMatrix(6, device="cuda"),
        ]

    g = torch.Generator(device="cuda").manual_seed(3)
    xs = [torch.randn(8, 6, device="cuda", generator=g) for _ in range(12)]
    ys = [torch.randint(0, 6, (8,), device="cuda", generator=g) for _ in range(12)]
    graphed, eager = five(), five()
    step = GraphedUpdate(graphed, xs[0], ys[0])
    assert step.direct_us > 0 and step.replay_us > 0
    for x, y in zip(xs, ys):
        assert step(x, y) is graphed
        for m in eager:
            m.update(x, y)
    for a, b in zip(graphed, eager):
        torch.testing.assert_close(a.compute(), b.compute())
    print(f"GraphedUpdate of 5 metrics bs=8: direct {step.direct_us:.1f} us, replay {step.replay_us:.1f} us")
