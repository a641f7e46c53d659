import pytest
import torch
import torch.distributed as dist

from torcheval_amd.metrics import MulticlassAccuracy
from torcheval_amd.metrics.toolkit import (
    classwise_converter,
    clone_metric,
    clone_metrics,
    get_synced_metric,
    get_synced_metric_collection,
    get_synced_state_dict,
    get_synced_state_dict_collection,
    reset_metrics,
    sync_and_compute,
    sync_and_compute_collection,
    to_device,
)
from torcheval_amd.parallel import allreduce_coalesced, packed_all_gather
from torcheval_amd.utils.test_utils import (
    DummySumDictStateMetric,
    DummySumListStateMetric,
    DummySumMetric,
    run_distributed,
)


def _sync_dummies(rank, ws):
    s = DummySumMetric().update(torch.tensor(float(rank + 1)))
    lst = DummySumListStateMetric()
    for i in range(rank):  # rank 0 holds an EMPTY list
        lst.update(torch.arange(i + 1, dtype=torch.float32))
    d = DummySumDictStateMetric().update(f"k{rank % 2}", torch.tensor(float(rank)))
    acc = MulticlassAccuracy(average=None, num_classes=3)
    acc.update(torch.tensor([rank % 3]), torch.tensor([rank % 3]))
    single = sync_and_compute(s)
    coll = sync_and_compute_collection({"s": s, "l": lst, "d": d, "a": acc})
    sd = get_synced_state_dict(lst)
    sdc = get_synced_state_dict_collection({"s": s})
    synced = get_synced_metric(s)
    assert synced is not s
    torch.testing.assert_close(s.sum, torch.tensor(float(rank + 1)))  # local untouched
    return single, {k: (dict(v) if isinstance(v, dict) else v) for k, v in coll.items()}, len(sd["x"]), sdc


@pytest.mark.parametrize("ws", [2, 4])
def test_sync_and_compute_everywhere(ws):
    results = run_distributed(_sync_dummies, ws)
    total = float(sum(range(1, ws + 1)))
    for single, coll, nlist, sdc in results:
        torch.testing.assert_close(single, torch.tensor(total))
        torch.testing.assert_close(coll["s"], torch.tensor(total))
        exp_list = sum(float(torch.arange(i + 1).sum()) for r in range(ws) for i in range(r))
        torch.testing.assert_close(coll["l"], torch.tensor(exp_list))
        assert nlist == sum(range(ws))
        exp_d = {"k0": sum(r for r in range(ws) if r % 2 == 0), "k1": sum(r for r in range(ws) if r % 2 == 1)}
        assert {k: float(v) for k, v in coll["d"].items()} == {k: float(v) for k, v in exp_d.items()}
        torch.testing.assert_close(coll["a"], torch.ones(3) if ws >= 3 else torch.tensor([1.0, 1.0, float("nan")]), equal_nan=True)
        torch.testing.assert_close(sdc["s"]["sum"], torch.tensor(total))


def _collectives(rank, ws):
    a = torch.tensor([rank, -rank], dtype=torch.float32)
    b = torch.tensor([[rank]], dtype=torch.int64)
    c = torch.tensor([rank == 1, True])
    red = allreduce_coalesced([a, b, a, c], ["sum", "max", "min", "max"])
    tree = {"x": [torch.full((rank + 1,), rank, dtype=torch.float64)], "n": rank, "s": "r%d" % rank,
            "e": torch.empty(0, 3), "h": torch.ones(2, dtype=torch.bfloat16) * rank}
    g = packed_all_gather(tree)
    return red, g


def test_collectives_gloo():
    res = run_distributed(_collectives, 3)
    for red, g in res:
        torch.testing.assert_close(red[0], torch.tensor([3.0, -3.0]))
        assert red[1].item() == 2
        torch.testing.assert_close(red[2], torch.tensor([0.0, -2.0]))
        assert red[3].tolist() == [True, True]
        for r in range(3):
            assert g[r]["n"] == r and g[r]["s"] == "r%d" % r
            torch.testing.assert_close(g[r]["x"][0], torch.full((r + 1,), r, dtype=torch.float64))
            assert g[r]["e"].shape == (0, 3)
            torch.testing.assert_close(g[r]["h"], torch.ones(2, dtype=torch.bfloat16) * r)


def test_world_size_one_returns_input():
    m = DummySumMetric()
    assert get_synced_metric(m) is m
    coll = {"m": m}
    assert get_synced_metric_collection(coll) is coll
    torch.testing.assert_close(sync_and_compute(m), torch.tensor(0.0))


def test_clone_reset_to_device():
    m = DummySumMetric().update(torch.tensor(2.0))
    c = clone_metric(m)
    c.update(torch.tensor(1.0))
    torch.testing.assert_close(m.sum, torch.tensor(2.0))
    cs = clone_metrics([m, m])
    assert len(cs) == 2 and cs[0] is not m
    reset_metrics([m])
    torch.testing.assert_close(m.sum, torch.tensor(0.0))
    (m2,) = to_device([m], torch.device("cpu"))
    assert m2.device == torch.device("cpu")


def test_classwise_converter():
    x = torch.tensor([0.1, 0.2])
    assert set(classwise_converter(x, "acc")) == {"acc_0", "acc_1"}
    assert set(classwise_converter(x, "acc", ["a", "b"])) == {"acc_a", "acc_b"}
    with pytest.raises(ValueError, match="Number of labels 3 must be equal"):
        classwise_converter(x, "acc", ["a", "b", "c"])


def _async_sync(rank, ws):
    from torcheval_amd.metrics import BinaryAUROC, WindowedClickThroughRate
    from torcheval_amd.metrics.toolkit import get_synced_metric_async, sync_and_compute_async

    acc = MulticlassAccuracy()
    acc.update(torch.tensor([[0.9, 0.1], [0.2, 0.8]]), torch.tensor([0, rank % 2]))  # typed (sum)
    auroc = BinaryAUROC()
    auroc.update(torch.tensor([0.1 * (rank + 1), 0.5]), torch.tensor([rank % 2, 1]))  # typed (cat)
    ctr = WindowedClickThroughRate(max_num_updates=2)
    ctr.update(torch.tensor([1, 0, rank % 2]))  # untyped (window merge)
    expect_acc = sync_and_compute(acc)
    expect_auroc = sync_and_compute(auroc)
    expect_ctr = sync_and_compute(ctr)
    fut = sync_and_compute_async({"acc": acc, "auroc": auroc, "ctr": ctr})
    single = get_synced_metric_async(acc)
    # keep updating while the sync is in flight: must not leak into the result
    for _ in range(3):
        acc.update(torch.tensor([[0.0, 1.0]]), torch.tensor([0]))
        auroc.update(torch.tensor([0.99]), torch.tensor([0]))
        ctr.update(torch.tensor([0, 0, 0]))
    res = fut.compute()
    torch.testing.assert_close(res["acc"], expect_acc)
    torch.testing.assert_close(res["auroc"], expect_auroc)
    torch.testing.assert_close(res["ctr"][0], expect_ctr[0])
    torch.testing.assert_close(res["ctr"][1], expect_ctr[1])
    torch.testing.assert_close(single.compute(), expect_acc)
    assert float(acc.num_total) == 5.0  # the live metric kept its local updates
    return True


@pytest.mark.parametrize("ws", [2, 3])
def test_async_sync_snapshots_states(ws):
    assert all(run_distributed(_async_sync, ws))


def test_async_sync_world_size_one():
    from torcheval_amd.metrics.toolkit import sync_and_compute_async

    m = MulticlassAccuracy().update(torch.tensor([[0.9, 0.1]]), torch.tensor([0]))
    fut = sync_and_compute_async(m)
    m.update(torch.tensor([[0.9, 0.1]]), torch.tensor([1]))
    torch.testing.assert_close(fut.compute(), torch.tensor(1.0))
