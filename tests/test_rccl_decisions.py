"""The multi-rank decisions of the direct-RCCL engine (parallel/rccl_direct.py), driven over 2-4
gloo CPU ranks with a fake native layer (no GPU): every rank must take the same path - direct
communicator or torch.distributed - and no rank may hang, when

* communicator init fails on one rank only,
* the bootstrap self-check fails on one rank only,
* one rank's watchdog marks its communicator failed mid-run (async error handling off: the
  group votes before the next sync and every rank rebuilds at that same sync).

The fake's "direct" collectives run over a separate gloo group, so a rank that skips a
collective its peers entered hangs them exactly as a real communicator would; the pool's job
timeout turns such a hang into a failure.  Replaces the decision points around reference
torcheval/metrics/toolkit.py:371-391 (whose all_gather_object has no second communicator)."""

import os

import pytest
import torch

from torcheval_amd.utils.test_utils.dist_pool import run_distributed


class _FakeNative:
    """The rccl_* entry points rccl_direct.py calls, over a gloo group ``sub``."""

    def __init__(self, rank, ws, sub, fail_init_rank=-1, bad_check_rank=-1):
        self.rank, self.ws, self.sub = rank, ws, sub
        self.fail_init = rank == fail_init_rank
        self.bad_check = rank == bad_check_rank
        self.states = {}
        self.log = []

    def rccl_available(self):
        return True

    def rccl_unique_id(self, out):
        out.fill_(7)

    def rccl_comm_init(self, uid, ws, rank, device, timeout_ms):
        self.log.append("init")
        if self.fail_init:
            raise RuntimeError("fake: ncclCommInitRank failed")
        h = len(self.states)
        self.states[h] = 0
        return h

    def _usable(self, h):
        if self.states.get(h) != 0:
            raise RuntimeError(f"fake: communicator {h} is unusable")

    def rccl_all_reduce(self, h, t, op, out=None):
        import torch.distributed as dist

        self._usable(h)
        r = t.clone()
        dist.all_reduce(r, op={0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MAX, 2: dist.ReduceOp.MIN}[op], group=self.sub)
        if self.bad_check:
            r += 1
        (out if out is not None else t).copy_(r)

    def rccl_all_gather(self, h, src, out):
        import torch.distributed as dist

        self._usable(h)
        parts = [torch.empty_like(src) for _ in range(self.ws)]
        dist.all_gather(parts, src, group=self.sub)
        out.copy_(torch.cat(parts))

    def rccl_comm_state(self, h):
        return self.states.get(h, -1)

    def rccl_comm_destroy(self, h):
        self.log.append(f"destroy{h}")
        self.states[h] = 3

    def rccl_comm_abort(self, h):
        self.log.append(f"abort{h}")
        self.states[h] = 2

    def rccl_wait_aborted(self, h, timeout_ms):
        if self.states.get(h) == 1:  # the watchdog's background abort
            self.states[h] = 2
        return True


def _run_case(rank, ws, case):
    import torch.distributed as dist

    import torcheval_amd.ops as ops
    from torcheval_amd.parallel import rccl_direct as rd

    sub = dist.new_group(backend="gloo")  # the fake communicators' transport
    fake = _FakeNative(rank, ws, sub, fail_init_rank=1 if case == "init_fails_on_one_rank" else -1,
                       bad_check_rank=ws - 1 if case == "self_check_fails_on_one_rank" else -1)
    saved = (ops.native, ops.native_loaded, rd._DEVICE_TYPES, dict(os.environ))
    ops.native = lambda: fake
    ops.native_loaded = lambda: True
    rd._DEVICE_TYPES = ("cuda", "cpu")
    os.environ["TORCHEVAL_AMD_DIRECT_RCCL"] = "1"
    if case == "watchdog_fails_one_rank":
        os.environ["TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING"] = "0"
    rd._COMMS.clear()
    del rd._ABORTING[:]
    dev = torch.device("cpu")
    group = dist.group.WORLD
    out = {}
    try:
        h = rd.comm_for(group, ws, dev)
        out["direct"] = h is not None
        out["cached"] = rd.comm_for(group, ws, dev) == h  # no second bootstrap
        if case == "watchdog_fails_one_rank":
            x, r = torch.tensor([float(rank + 1)]), torch.empty(1)
            rd.all_reduce(h, x, "sum", r)  # sync 1 on the first communicator
            out["sum1"] = float(r)
            if rank == 1:
                fake.states[h] = 1  # this rank's watchdog fired; its peers saw nothing
            h2 = rd.agree(h, group, ws, dev)  # every rank votes before sync 2
            out["rebuilt"] = h2 is not None and h2 != h
            out["old_dropped"] = fake.states[h] in (2, 3)
            rd.all_reduce(h2, x, "sum", r)  # sync 2: every rank on the NEW communicator
            out["sum2"] = float(r)
            out["agree_again"] = rd.agree(h2, group, ws, dev) == h2  # healthy: no rebuild
        out["log"] = fake.log
        return out
    finally:
        ops.native, ops.native_loaded, rd._DEVICE_TYPES = saved[:3]
        os.environ.clear()
        os.environ.update(saved[3])
        rd._COMMS.clear()
        del rd._ABORTING[:]


@pytest.mark.parametrize("ws", [2, 3, 4])
def test_healthy_group_goes_direct_everywhere(ws):
    res = run_distributed(_run_case, ws, "healthy", timeout=60)
    assert all(r["direct"] and r["cached"] for r in res)
    assert all(r["log"] == ["init"] for r in res)


@pytest.mark.parametrize("ws", [2, 4])
def test_init_failure_on_one_rank_sends_every_rank_to_torch_distributed(ws):
    res = run_distributed(_run_case, ws, "init_fails_on_one_rank", timeout=60)
    assert not any(r["direct"] for r in res)  # the same path everywhere, nobody hung
    assert all(r["cached"] for r in res)  # the decision is cached: no re-bootstrap per sync
    for rank, r in enumerate(res):  # the ranks that did get a communicator released it
        assert r["log"] == (["init"] if rank == 1 else ["init", "destroy0"])


@pytest.mark.parametrize("ws", [3, 4])
def test_self_check_failure_on_one_rank_sends_every_rank_to_torch_distributed(ws):
    res = run_distributed(_run_case, ws, "self_check_fails_on_one_rank", timeout=60)
    assert not any(r["direct"] for r in res)
    assert all(r["log"] == ["init", "destroy0"] for r in res)


@pytest.mark.parametrize("ws", [2, 3])
def test_watchdog_failure_on_one_rank_rebuilds_on_every_rank(ws):
    res = run_distributed(_run_case, ws, "watchdog_fails_one_rank", timeout=60)
    want = float(ws * (ws + 1) // 2)
    for rank, r in enumerate(res):
        assert r["direct"] and r["sum1"] == want
        assert r["rebuilt"] and r["old_dropped"] and r["sum2"] == want and r["agree_again"]
        # the failed rank waited for its watchdog's abort; its peers aborted their healthy copy
        assert r["log"][:2] == ["init", "init"] or r["log"] == ["init", "abort0", "init"]
        assert ("abort0" in r["log"]) == (rank != 1)


def test_default_policy_keeps_multi_rank_groups_on_torch_distributed(monkeypatch):
    from torcheval_amd.parallel import rccl_direct as rd

    monkeypatch.delenv("TORCHEVAL_AMD_DIRECT_RCCL", raising=False)
    assert not rd.enabled(2) and not rd.enabled(8)
    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "0")
    assert not rd.enabled(1)


def test_deterministic_flag_keeps_multi_rank_groups_rank_ordered(monkeypatch):
    from torcheval_amd.config import flags
    from torcheval_amd.parallel import rccl_direct as rd

    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "1")
    with flags(deterministic=True):
        assert not rd.enabled(2) and not rd.enabled(8)
