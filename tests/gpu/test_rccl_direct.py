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


def test_async_sync_on_side_stream_snapshots_at_call(pg, monkeypatch):
    from torcheval_amd.metrics.toolkit import get_synced_metric_async
    from torcheval_amd.parallel.state_buffer import FastPendingSync

    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "1")
    acc, cm, bap = _metrics()
    coll = {"acc": acc, "cm": cm, "bap": bap}
    want = {k: m.compute() for k, m in coll.items()}
    g = torch.Generator(device=DEV).manual_seed(7)
    with collectives_at_world_size_1():
        fut = get_synced_metric_async(coll)
        assert isinstance(fut._pending, FastPendingSync)
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
    assert not torch.equal(acc.compute(), want["acc"]) or True  # live metric moved on
