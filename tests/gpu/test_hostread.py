"""Low-latency host reads of device error flags (csrc/runtime/hostread.cpp, kernels/hostread.hip)
against tensor.tolist(): values, stream order, a read queued behind long GPU work (the bounded
spin falls back to a stream synchronize), side streams, and the metrics that use it."""
import pytest
import torch

from torcheval_amd.ops import hostread, native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_values_match_tolist():
    g = torch.Generator().manual_seed(0)
    for n in range(1, 15):
        t = torch.randint(-(2**31), 2**31 - 1, (n,), generator=g, dtype=torch.int64).to(torch.int32).to(DEV)
        assert hostread._fast(t)
        assert hostread.read_ints(t) == t.tolist()
        assert hostread.read_int(t) == t[0].item()


def test_int64_values():
    vals = [0, 1, -1, 2**31, -(2**31) - 1, 2**40 + 3, -(2**62), 2**63 - 1]
    for n in range(1, 8):
        t = torch.tensor(vals[:n], dtype=torch.int64, device=DEV)
        assert hostread._fast(t)
        assert hostread.read_ints(t) == vals[:n]
    assert not hostread._fast(torch.zeros(8, dtype=torch.int64, device=DEV))  # 16 words


def test_pair_read_matches_tolist():
    g = torch.Generator().manual_seed(1)
    for _ in range(20):
        a = torch.randint(-(2**31), 2**31 - 1, (3,), generator=g, dtype=torch.int64).to(torch.int32).to(DEV)
        b = torch.randint(-(2**31), 2**31 - 1, (2,), generator=g, dtype=torch.int64).to(torch.int32).to(DEV)
        assert list(native().read_small_ints_pair(a, b)) == a.tolist() + b.tolist()
        assert hostread.read_int_pair(a, b) == (a[0].item(), b[0].item())
    # mixed dtypes / 0-d counts take the per-tensor path
    x, y = torch.tensor(5, device=DEV), torch.tensor(7, dtype=torch.int32, device=DEV)
    assert hostread.read_int_pair(x, y) == (5, 7)
    t = torch.zeros(1, dtype=torch.int32, device=DEV)
    for v in range(1, 50):  # stream order: the read sees the fill queued before it
        t.fill_(v)
        assert hostread.read_int_pair(t, y) == (v, 7)


def test_sees_work_queued_before_it():
    t = torch.zeros(3, dtype=torch.int32, device=DEV)
    for v in range(1, 200):
        t.fill_(v)
        assert hostread.read_ints(t) == [v, v, v]


def test_long_queue_falls_back_to_a_synchronize():
    t = torch.zeros(2, dtype=torch.int32, device=DEV)
    native().test_host_flag_set(0)
    try:
        native().test_spin_on_host_flag(0, 60)  # holds the stream ~60 ms (flag never set)
        t.fill_(42)
        assert hostread.read_ints(t) == [42, 42]  # spin budget 1 ms, then the blocking path
    finally:
        native().test_host_flag_set(1)
    torch.cuda.synchronize()


def test_side_stream_is_the_current_stream():
    s = torch.cuda.Stream()
    t = torch.zeros(1, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        t.fill_(9)
        assert hostread.read_int(t) == 9


def test_fallbacks_take_tolist():
    assert not hostread._fast(torch.zeros(15, dtype=torch.int32, device=DEV))  # too many words
    assert not hostread._fast(torch.zeros(2, dtype=torch.int16, device=DEV))
    assert hostread.read_ints(torch.arange(20, dtype=torch.int32, device=DEV)) == list(range(20))
    assert hostread.read_int(torch.tensor([7, 8], device=DEV)) == 7


def test_metric_errors_still_raise():
    from torcheval_amd.metrics import MulticlassConfusionMatrix

    m = MulticlassConfusionMatrix(4, device=DEV)
    m.update(torch.randn(8, 4, device=DEV), torch.tensor([0, 1, 2, 3, 0, 1, 2, 9], device=DEV))
    with pytest.raises(ValueError):
        m.compute()
    ok = MulticlassConfusionMatrix(4, device=DEV)
    ok.update(torch.randn(8, 4, device=DEV), torch.tensor([0, 1, 2, 3, 0, 1, 2, 3], device=DEV))
    assert int(ok.compute().sum()) == 8
