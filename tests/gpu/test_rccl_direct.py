"""Direct RCCL communicators (csrc/runtime/rccl_direct.cpp, parallel/rccl_direct.py) on a
1-rank ``nccl`` group: the primitives against torch, and the state-buffer sync through them
bit-equal to the torch.distributed path (``TORCHEVAL_AMD_DIRECT_RCCL=0``).
(Reference sync path: toolkit.py:371-391.)"""

import socket

import pytest
import torch
import torch.distributed as dist

from torcheval_amd.ops import native
from torcheval_amd.parallel import rccl_direct
from torcheval_amd.parallel.collectives import collectives_at_world_size_1

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def pg():
    if dist.is_initialized():
        pytest.skip("a default process group already exists in this process")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=DEV)
    yield dist.group.WORLD
    dist.destroy_process_group()


def test_library_resolved():
    assert native().rccl_available()


def test_primitives(pg):
    h = rccl_direct.comm_for(pg, 1, DEV)
    assert h is not None and rccl_direct.comm_for(pg, 1, DEV) == h  # cached per group
    src = torch.arange(37, dtype=torch.uint8, device=DEV)
    out = torch.empty(37, dtype=torch.uint8, device=DEV)
    rccl_direct.all_gather(h, src, out)
    assert torch.equal(out, src)
    for dtype in (torch.float32, torch.float64, torch.int64, torch.int32):
        t = (torch.randn(1001, device=DEV) * 100).to(dtype)
        ref = t.clone()
        for op in ("sum", "max", "min"):
            rccl_direct.all_reduce(h, t, op)
            assert torch.equal(t, ref)  # one rank: every reduction is the identity
    o = torch.full((1001,), -1.0, device=DEV)
    s_ = torch.randn(1001, device=DEV)
    rccl_direct.all_reduce(h, s_, "sum", out=o)  # out of place: the send buffer is untouched
    assert torch.equal(o, s_)
    # dispatcher forms
    torch.ops.torcheval_amd.rccl_all_gather(h, src, out)
    torch.ops.torcheval_amd.rccl_all_reduce(h, t, 0)
    torch.cuda.synchronize()
    assert rccl_direct._self_check(h, 1, 0, torch.device(DEV))  # the ws > 1 bootstrap check's calls


def test_accuracy_plan_uses_one_all_reduce(pg):
    from torcheval_amd.metrics.toolkit import sync_and_compute
    from torcheval_amd.parallel import state_buffer as sbm

    acc, _, _ = _metrics()
    with collectives_at_world_size_1():
        v = sync_and_compute(acc)
        plan = sbm._plan_for(sbm.buffer_of(acc), dist.group.WORLD, 1, acc)
    assert plan.single is not None and plan.comm is not None
    assert torch.equal(v, acc.compute())


def _metrics():
    from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix, BinaryBinnedAUPRC

    g = torch.Generator(device=DEV).manual_seed(0)
    acc = MulticlassAccuracy(device=DEV)
    cm = MulticlassConfusionMatrix(100, device=DEV)
    bap = BinaryBinnedAUPRC(threshold=50, device=DEV)
    for _ in range(3):
        x = torch.randn(4096, 100, device=DEV, generator=g)
        y = torch.randint(0, 100, (4096,), device=DEV, generator=g)
        acc.update(x, y)
        cm.update(x, y)
        bap.update(torch.rand(4096, device=DEV, generator=g), (y % 2))
    return acc, cm, bap


@pytest.mark.parametrize("direct", ["1", "0"])
def test_sync_matches_torch_distributed(pg, monkeypatch, direct):
    from torcheval_amd.metrics.toolkit import sync_and_compute

    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", direct)
    acc, cm, bap = _metrics()
    with collectives_at_world_size_1():
        got = [sync_and_compute(m) for m in (acc, cm, bap)]
    want = [m.compute() for m in (acc, cm, bap)]
    for g_, w_ in zip(got, want):
        if isinstance(g_, tuple):
            for a, b in zip(g_, w_):
                assert torch.equal(a, b)
        else:
            assert torch.equal(g_, w_)


@pytest.mark.parametrize("direct", ["1", "0"])
def test_collection_sync_matches_local(pg, monkeypatch, direct):
    from torcheval_amd.metrics.toolkit import sync_and_compute_collection

    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", direct)
    acc, cm, bap = _metrics()
    coll = {"acc": acc, "cm": cm, "bap": bap}
    with collectives_at_world_size_1():
        got = sync_and_compute_collection(coll)
    for k, m in coll.items():
        w = m.compute()
        g_ = got[k]
        if isinstance(w, tuple):
            for a, b in zip(g_, w):
                assert torch.equal(a, b)
        else:
            assert torch.equal(g_, w)


@pytest.mark.parametrize("side_stream", ["1", "0"])
def test_async_sync_on_side_stream_snapshots_at_call(pg, monkeypatch, side_stream):
    """Async sync: the opt-in side-stream direct path and the default general engine (one
    communicator: torch.distributed's async collectives) both snapshot at the call."""
    from torcheval_amd.metrics.toolkit import get_synced_metric_async
    from torcheval_amd.parallel.state_buffer import FastPendingSync

    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "1")
    monkeypatch.setenv("TORCHEVAL_AMD_ASYNC_DIRECT_RCCL", side_stream)
    acc, cm, bap = _metrics()
    coll = {"acc": acc, "cm": cm, "bap": bap}

    def snap(v):  # compute() may hand out the live state (the reference's aliasing)
        return tuple(x.clone() for x in v) if isinstance(v, tuple) else v.clone()

    want = {k: snap(m.compute()) for k, m in coll.items()}
    g = torch.Generator(device=DEV).manual_seed(7)
    with collectives_at_world_size_1():
        fut = get_synced_metric_async(coll)
        assert isinstance(fut._pending, FastPendingSync) == (side_stream == "1")
        for _ in range(20):  # the live metrics keep changing while the collectives run
            x = torch.randn(4096, 100, device=DEV, generator=g)
            y = torch.randint(0, 100, (4096,), device=DEV, generator=g)
            acc.update(x, y)
            cm.update(x, y)
        synced = fut.wait()
    for k, w in want.items():
        got = synced[k].compute()
        if isinstance(w, tuple):
            for a, b in zip(got, w):
                assert torch.equal(a, b)
        else:
            assert torch.equal(got, w)
    # the live metrics moved on (20 more batches) while the synced copies kept the call's state
    assert float(acc.num_total) == 23 * 4096
    assert float(synced["acc"].num_total) == 3 * 4096
    assert float(cm.confusion_matrix.sum()) == 23 * 4096
    assert float(synced["cm"].confusion_matrix.sum()) == 3 * 4096


def test_graphed_update_survives_a_sync(pg):
    """a sync must not rebind the states a captured HIP graph writes."""
    from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.toolkit import get_synced_metric, sync_and_compute
    from torcheval_amd.utils.graphs import GraphedUpdate

    g = torch.Generator(device=DEV).manual_seed(3)
    xs = [torch.randn(1024, 50, device=DEV, generator=g) for _ in range(5)]
    ys = [torch.randint(0, 50, (1024,), device=DEV, generator=g) for _ in range(5)]
    for m in (MulticlassAccuracy(device=DEV), MulticlassConfusionMatrix(50, device=DEV)):
        step = GraphedUpdate(m, xs[0], ys[0])
        for i in range(3):
            step(xs[i], ys[i])
        with collectives_at_world_size_1():
            synced = get_synced_metric(m)
            v = sync_and_compute(m)
        torch.testing.assert_close(v, synced.compute())
        for i in range(3, 5):
            step(xs[i], ys[i])  # must land in the live metric
        ref = type(m)(device=DEV) if isinstance(m, MulticlassAccuracy) else MulticlassConfusionMatrix(50, device=DEV)
        for i in range(5):
            ref.update(xs[i], ys[i])
        assert torch.equal(m.compute(), ref.compute())
        m.reset()  # in place: the graph keeps writing the same buffer
        step(xs[0], ys[0])
        ref.reset()
        ref.update(xs[0], ys[0])
        assert torch.equal(m.compute(), ref.compute())
        m.load_state_dict(ref.state_dict())  # rebinds: the next replay must refuse
        with pytest.raises(RuntimeError, match="rebound after graph capture"):
            step(xs[1], ys[1])


def test_direct_plan_covers_flags_bool_and_wide_types(pg):
    """The out-of-place grouped plan: confusion matrix (large f32 group + int32 flag), bool /
    f64 / i64 states; the synced copies view a fresh buffer, the live buffer is untouched."""
    from torcheval_amd.metrics.toolkit import get_synced_metric
    from torcheval_amd.parallel import state_buffer as sbm
    from torcheval_amd.metrics.metric import Metric

    class Mixed(Metric[torch.Tensor]):
        def __init__(self):
            super().__init__(device=DEV)
            self._add_state("f", torch.zeros(5, dtype=torch.float64, device=DEV), merge="sum")
            self._add_state("i", torch.zeros(3, dtype=torch.int64, device=DEV), merge="max")
            self._add_state("b", torch.zeros(7, dtype=torch.bool, device=DEV), merge="sum")
            self._add_state("h", torch.zeros(9, dtype=torch.bfloat16, device=DEV), merge="min")

        def update(self, x):
            self.f += x[:5].double()
            self.i.copy_(torch.maximum(self.i, x[:3].long()))
            self.b |= x[:7] > 0
            self.h.copy_(torch.minimum(self.h, x[:9].bfloat16()))
            return self

        def compute(self):
            return self.f

        def merge_state(self, metrics):
            return self

    _, cm, _ = _metrics()
    mx = Mixed().update(torch.arange(-4.0, 12.0, device=DEV))
    with collectives_at_world_size_1():
        for m in (cm, mx):
            synced = get_synced_metric(m)
            plan = sbm._plan_for(sbm.buffer_of(m), dist.group.WORLD, 1, m)
            assert plan.rplan is not None
            for name in m._state_merge_kinds():
                a, b = getattr(synced, name), getattr(m, name)
                assert torch.equal(a, b) and a.data_ptr() != b.data_ptr(), name
    assert synced.b.dtype == torch.bool
    assert torch.equal(get_synced_metric_flag(cm), torch.zeros(3, dtype=torch.int32, device=DEV))


def get_synced_metric_flag(cm):
    from torcheval_amd.metrics.toolkit import get_synced_metric

    with collectives_at_world_size_1():
        return get_synced_metric(cm)._err


def test_sync_timeout_raises_then_recovers(pg):
    """A collective held behind a spinning kernel: ``timeout=`` raises TimeoutError near the
    deadline (direct path kept), the communicator is aborted in the background, and the next
    sync builds a fresh one and succeeds."""
    import time
    from datetime import timedelta

    from torcheval_amd.metrics.toolkit import sync_and_compute

    _, cm, _ = _metrics()
    with collectives_at_world_size_1():
        want = sync_and_compute(cm)  # builds the communicator and the plan
        torch.cuda.synchronize()
        h_old = rccl_direct.comm_for(dist.group.WORLD, 1, DEV)
        native().test_host_flag_set(0)
        native().test_spin_on_host_flag(0, 20000)  # holds the stream for at most 20 s
        t0 = time.perf_counter()
        raised = None
        try:
            try:
                sync_and_compute(cm, timeout=timedelta(milliseconds=500))
            except TimeoutError as e:
                raised = e
            elapsed = time.perf_counter() - t0
        finally:
            native().test_host_flag_set(1)
        if raised is None:
            from torcheval_amd.parallel.state_buffer import plan_summary

            sb = cm.__dict__.get("_tea_sb")
            plans = [(k, p.comm, p.rplan, p.gen) for k, p in sb.plans.items()] if sb is not None else None
            pytest.fail(f"no TimeoutError after {elapsed:.3f} s; comm {h_old} state {rccl_direct.state(h_old)}; "
                        f"plan {plan_summary(cm)}; plans {plans} gen {rccl_direct.GENERATION[0]}; "
                        f"comm now {rccl_direct.comm_for(dist.group.WORLD, 1, DEV)}")
        assert "did not complete" in str(raised)
        torch.cuda.synchronize()
        assert 0.4 < elapsed < 5.0, elapsed
        assert rccl_direct.state(h_old) in (1, 2)
        got = sync_and_compute(cm, timeout=timedelta(seconds=60))
        h_new = rccl_direct.comm_for(dist.group.WORLD, 1, DEV)
    assert h_new != h_old and rccl_direct.state(h_new) == 0
    assert rccl_direct.state(h_old) == 2  # aborted
    assert torch.equal(got, want)


def test_watchdog_deadline_without_timeout_argument(pg, monkeypatch):
    """No ``timeout=``: the sync returns at once (stream-ordered) and the watchdog enforces the
    communicator's deadline (the process group's timeout by default) in the background.  With
    TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING=0 the process survives; the next sync rebuilds."""
    import time

    from torcheval_amd.metrics.toolkit import get_synced_metric, sync_and_compute

    monkeypatch.setenv("TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING", "0")
    acc, _, _ = _metrics()
    with collectives_at_world_size_1():
        want = sync_and_compute(acc)
        torch.cuda.synchronize()
        h = rccl_direct.comm_for(dist.group.WORLD, 1, DEV)
        assert rccl_direct.group_timeout(dist.group.WORLD, DEV).total_seconds() > 60  # the PG's own
        native().rccl_set_timeout(h, 300)
        native().test_host_flag_set(0)
        native().test_spin_on_host_flag(0, 20000)
        try:
            fut = get_synced_metric(acc)  # enqueued behind the spinning kernel; no host wait
            deadline = time.perf_counter() + 10
            while rccl_direct.state(h) == 0 and time.perf_counter() < deadline:
                time.sleep(0.05)
            st = rccl_direct.state(h)
        finally:
            native().test_host_flag_set(1)
        torch.cuda.synchronize()
        del fut
        assert st in (1, 2), st
        assert "did not complete" in native().rccl_comm_reason(h)
        # the failure was not observed by a waiter: the next use raises (its result would have
        # been garbage), and the sync after that runs on a fresh communicator
        with pytest.raises(RuntimeError, match="unusable"):
            sync_and_compute(acc)
        assert native().rccl_wait_aborted(h, 30000)
        got = sync_and_compute(acc)
        assert rccl_direct.comm_for(dist.group.WORLD, 1, DEV) != h
    assert torch.equal(got, want)
