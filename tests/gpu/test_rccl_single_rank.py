"""RCCL code paths on one MI355X: a 1-rank ``nccl`` (= RCCL) process group in this process.

Every collective branch that the gloo CPU tests cannot reach runs here for real on HBM
tensors: ``all_gather_into_tensor`` (packed all-gather-v header + payload, error flags),
bucketed ``all_reduce``, ``reduce_scatter_tensor`` (class sharding) and ``all_to_all_single``
(sample-sharded AUROC).  ``collectives_at_world_size_1`` disables the ws == 1 shortcuts so the
multi-rank code runs with one rank; each result must equal the local compute.
(Reference sync path: toolkit.py:371-391.)
"""

import socket

import pytest
import torch
import torch.distributed as dist

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
    dist.init_process_group(
        "nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
        device_id=DEV,
    )
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.destroy_process_group()


def test_transport_is_hbm(pg):
    from torcheval_amd.parallel.distributed import backend_of, transport_device

    assert backend_of(pg) == "nccl"
    assert transport_device(pg).type == "cuda"


def test_allreduce_coalesced_rccl(pg):
    from torcheval_amd.parallel.collectives import allreduce_coalesced, allreduce_coalesced_async

    a = torch.randn(1000, device=DEV)
    b = torch.randint(-5, 5, (7, 3), device=DEV)
    c = torch.tensor([True, False], device=DEV)
    h = allreduce_coalesced_async([a, b, a, c, b], ["sum", "max", "min", "max", "sum"], pg)
    a.add_(1.0)  # the packing copy snapshotted the state already
    out = h.wait()
    torch.testing.assert_close(out[0], a - 1.0)
    torch.testing.assert_close(out[1], b)
    assert out[3].dtype == torch.bool and out[3].tolist() == [True, False]
    assert all(t.is_cuda for t in out)
    # many tensors, tiny bucket cap: several buckets in flight at once
    ts = [torch.full((100,), float(i), device=DEV) for i in range(10)]
    res = allreduce_coalesced(ts, ["sum"] * 10, pg, bucket_cap_bytes=1000)
    for i, r in enumerate(res):
        torch.testing.assert_close(r, ts[i])


def test_packed_all_gather_rccl(pg):
    from torcheval_amd.parallel.collectives import _all_gather_fixed, packed_all_gather

    tree = {"x": [torch.arange(5, dtype=torch.float64, device=DEV)], "n": 3, "s": "r0",
            "e": torch.empty(0, 3, device=DEV), "h": torch.ones(17, dtype=torch.bfloat16, device=DEV),
            "b": torch.tensor([True, False, True], device=DEV)}
    g = packed_all_gather(tree, pg, 1)
    assert len(g) == 1 and g[0]["n"] == 3 and g[0]["s"] == "r0"
    torch.testing.assert_close(g[0]["x"][0], tree["x"][0])
    assert g[0]["x"][0].is_cuda  # never left HBM
    assert g[0]["e"].shape == (0, 3)
    torch.testing.assert_close(g[0]["h"], tree["h"])
    assert g[0]["b"].tolist() == [True, False, True]
    flat = _all_gather_fixed(torch.arange(4, device=DEV), pg, 1)
    assert flat.tolist() == [0, 1, 2, 3]


def _local_and_synced(metric, fn=None):
    from torcheval_amd.metrics.toolkit import get_synced_metric

    with collectives_at_world_size_1():
        synced = get_synced_metric(metric)
    assert synced is not metric
    f = fn or (lambda m: m.compute())
    return f(metric), f(synced)


def test_sync_typed_metrics_rccl(pg):
    from torcheval_amd.metrics import (
        BinaryAUROC,
        MulticlassAccuracy,
        MulticlassConfusionMatrix,
        Max,
        Min,
    )

    x = torch.randn(4096, 100, device=DEV)
    y = torch.randint(0, 100, (4096,), device=DEV)
    for m in (MulticlassAccuracy(device=DEV), MulticlassAccuracy(average="macro", num_classes=100, device=DEV),
              MulticlassConfusionMatrix(100, device=DEV)):
        m.update(x, y)
        a, b = _local_and_synced(m)
        torch.testing.assert_close(a, b)
    au = BinaryAUROC(device=DEV)
    for _ in range(3):
        au.update(torch.rand(10_000, device=DEV), torch.randint(0, 2, (10_000,), device=DEV))
    a, b = _local_and_synced(au)
    torch.testing.assert_close(a, b)
    for cls in (Max, Min):
        m = cls(device=DEV).update(torch.randn(1000, device=DEV))
        a, b = _local_and_synced(m)
        torch.testing.assert_close(a, b)


def test_sync_untyped_metrics_rccl(pg):
    from torcheval_amd.metrics import WindowedClickThroughRate
    from torcheval_amd.utils.test_utils import DummySumDictStateMetric, DummySumListStateMetric

    ctr = WindowedClickThroughRate(max_num_updates=3, device=DEV)
    for i in range(5):
        ctr.update(torch.randint(0, 2, (64,), device=DEV))
    a, b = _local_and_synced(ctr)
    torch.testing.assert_close(a[0], b[0])
    torch.testing.assert_close(a[1], b[1])
    d = DummySumDictStateMetric(device=DEV).update("k", torch.tensor(2.0, device=DEV))
    a, b = _local_and_synced(d)
    assert {k: float(v) for k, v in a.items()} == {k: float(v) for k, v in b.items()}
    lst = DummySumListStateMetric(device=DEV).update(torch.arange(4.0, device=DEV))
    a, b = _local_and_synced(lst)
    torch.testing.assert_close(a, b)


def test_sync_collection_and_async_rccl(pg):
    from torcheval_amd.metrics import MulticlassAccuracy, Mean
    from torcheval_amd.metrics.toolkit import sync_and_compute_async, sync_and_compute_collection

    acc = MulticlassAccuracy(device=DEV).update(torch.randn(512, 10, device=DEV),
                                                torch.randint(0, 10, (512,), device=DEV))
    mean = Mean(device=DEV).update(torch.randn(512, device=DEV))
    want = {"acc": acc.compute(), "mean": mean.compute()}
    with collectives_at_world_size_1():
        got = sync_and_compute_collection({"acc": acc, "mean": mean})
        fut = sync_and_compute_async({"acc": acc, "mean": mean})
        acc.update(torch.randn(512, 10, device=DEV), torch.zeros(512, dtype=torch.long, device=DEV))
        got_async = fut.compute()
    for k in want:
        torch.testing.assert_close(got[k], want[k])
        torch.testing.assert_close(got_async[k], want[k])


def test_error_flags_travel_rccl(pg):
    from torcheval_amd.metrics import MulticlassAccuracy

    m = MulticlassAccuracy(num_classes=10, average="macro", device=DEV)
    m.update(torch.randn(64, 10, device=DEV), torch.full((64,), 12, dtype=torch.long, device=DEV))
    from torcheval_amd.metrics.toolkit import get_synced_metric

    with collectives_at_world_size_1():
        synced = get_synced_metric(m)
    assert synced._err is not m._err
    with pytest.raises(RuntimeError, match="index out of bounds|out of|num_classes"):
        synced.compute()
    with pytest.raises(RuntimeError):
        m.compute()  # the caller's own flag was not consumed by the synced copy


def test_reduce_scatter_classes_rccl(pg):
    from torcheval_amd.metrics import MulticlassBinnedAUPRC, MulticlassConfusionMatrix
    from torcheval_amd.parallel.class_shard import (
        class_sharded_compute,
        reduce_scatter_classes,
        sharded_confusion_matrix,
    )

    t = torch.randn(37, 5, device=DEV)
    with collectives_at_world_size_1():
        shard, start, stop = reduce_scatter_classes(t, dim=0, group=pg)
        assert (start, stop) == (0, 37)
        torch.testing.assert_close(shard, t)
        shard1, _, _ = reduce_scatter_classes(t, dim=1, group=pg)
        torch.testing.assert_close(shard1, t.t())

        x = torch.rand(20_000, 50, device=DEV)
        y = torch.randint(0, 50, (20_000,), device=DEV)
        b = MulticlassBinnedAUPRC(num_classes=50, threshold=64, average=None, device=DEV).update(x, y)
        torch.testing.assert_close(class_sharded_compute(b, group=pg), b.compute())
        cm = MulticlassConfusionMatrix(50, device=DEV).update(x, y)
        torch.testing.assert_close(class_sharded_compute(cm, group=pg), cm.compute())
        for norm in ("true", "pred", "all"):
            cmn = MulticlassConfusionMatrix(50, normalize=norm, device=DEV).update(x, y)
            rows = sharded_confusion_matrix(cmn, group=pg)
            torch.testing.assert_close(rows.gather(pg), cmn.compute().float(), rtol=1e-5, atol=1e-6)


def test_sample_sharded_auc_rccl(pg):
    from torcheval_amd.metrics import BinaryAUROC
    from torcheval_amd.metrics.functional import binary_auprc, binary_auroc
    from torcheval_amd.parallel.dist_auc import distributed_binary_areas, sharded_compute

    x = (torch.randint(0, 1000, (200_001,), device=DEV).float() / 1000)
    t = torch.randint(0, 2, (200_001,), device=DEV)
    w = torch.rand(200_001, device=DEV, dtype=torch.float64)
    with collectives_at_world_size_1():
        roc, pr = distributed_binary_areas(x, t, group=pg)
        torch.testing.assert_close(roc, binary_auroc(x, t).double(), rtol=1e-9, atol=1e-12)
        torch.testing.assert_close(pr.float(), binary_auprc(x, t), rtol=1e-5, atol=1e-6)
        rocw, _ = distributed_binary_areas(x, t, w, group=pg)
        torch.testing.assert_close(rocw, binary_auroc(x, t, weight=w).double(), rtol=1e-9, atol=1e-12)
        m = BinaryAUROC(device=DEV).update(x, t)
        torch.testing.assert_close(sharded_compute(m, group=pg), m.compute().double(), rtol=1e-9, atol=1e-12)


def test_sorted_run_sync_rccl(pg):
    """The synced BinaryAUROC / BinaryAUPRC arrive as sorted runs and merge (K3m) on HBM."""
    from torcheval_amd.metrics import BinaryAUPRC, BinaryAUROC
    from torcheval_amd.metrics.toolkit import get_synced_metric

    x = torch.randint(0, 300, (50_000,), device=DEV).float() / 300
    t = torch.randint(0, 2, (50_000,), device=DEV)
    roc = BinaryAUROC(device=DEV)
    pr = BinaryAUPRC(device=DEV)
    for lo in range(0, 50_000, 10_000):
        roc.update(x[lo:lo + 10_000], t[lo:lo + 10_000])
        pr.update(x[lo:lo + 10_000], t[lo:lo + 10_000])
    want_roc, want_pr = roc.compute(), pr.compute()
    with collectives_at_world_size_1():
        s_roc, s_pr = get_synced_metric(roc), get_synced_metric(pr)
    assert s_roc._sorted_runs and s_pr._sorted_runs
    torch.testing.assert_close(s_roc.compute(), want_roc, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(s_pr.compute(), want_pr, rtol=1e-6, atol=1e-6)
