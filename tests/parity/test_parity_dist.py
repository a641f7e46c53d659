"""Distributed differential parity: every class case of ``cases.py`` synced across gloo ranks
with ``sync_and_compute`` must reproduce the reference's own result.

* 2 ranks, each holding one contiguous half of the updates: ``sync_and_compute`` is
  ``clone(rank0).merge_state([rank1])`` on every rank, i.e. exactly the reference's "merged"
  golden (window metrics included: their merge concatenates windows).
* 4 ranks, one update each: compared with the reference's single-metric result wherever the
  reference's own merge is order/partition-invariant (golden full == golden merged).

Reference call stack being matched: toolkit.py:206-260 (all_gather_object + merge_state);
ours goes through typed RCCL/gloo buckets (parallel/state_sync.py) instead.
"""

import os
import sys
import warnings

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import cases  # noqa: E402
from test_parity import GOLDEN, KNOWN_DEVIATIONS, assert_same  # noqa: E402

from torcheval_amd.utils.test_utils import run_distributed  # noqa: E402


def _skip_reason(cid):
    for prefix, reason in KNOWN_DEVIATIONS.items():
        if cid.startswith(prefix):
            return reason
    return None


def _sync_all_cases(rank, world_size, empty_last_rank=False):
    import torcheval_amd.metrics as M
    from torcheval_amd.metrics.toolkit import sync_and_compute

    out = {}
    for cid, (cls_name, ctor, upd) in sorted(cases.CLASS.items()):
        updates = upd(cases.cid_seed(cid))
        if empty_last_rank:  # every update on ranks 0 .. ws-2, the last rank holds nothing
            per = -(-len(updates) // (world_size - 1))
            mine = [] if rank == world_size - 1 else updates[rank * per:(rank + 1) * per]
        else:
            per = len(updates) // world_size
            mine = updates[rank * per:(rank + 1) * per]
        m = getattr(M, cls_name)(**ctor())
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                for args, kwargs in mine:
                    m.update(*args, **kwargs)
                out[cid] = sync_and_compute(m)
        except Exception as e:  # reported per case in the parent
            out[cid] = {"__raise__": type(e).__name__, "msg": str(e)}
    return out


def _same(a, b):
    try:
        assert_same(a, b)
        return True
    except AssertionError:
        return False


@pytest.fixture(scope="module")
def synced_2():
    return run_distributed(_sync_all_cases, 2)


@pytest.fixture(scope="module")
def synced_4():
    return run_distributed(_sync_all_cases, 4)


@pytest.fixture(scope="module")
def synced_3_with_empty_rank():
    return run_distributed(_sync_all_cases, 3, True)


@pytest.mark.parametrize("cid", sorted(cases.CLASS))
def test_sync_2_ranks_matches_reference_merge(cid, synced_2):
    if _skip_reason(cid):
        pytest.skip(_skip_reason(cid))
    exp = GOLDEN["class"][cid]["merged"]
    for rank, res in enumerate(synced_2):
        assert not (isinstance(res[cid], dict) and "__raise__" in res[cid]), res[cid]
        assert_same(res[cid], exp, f"rank{rank}")


@pytest.mark.parametrize("cid", sorted(cases.CLASS))
def test_sync_4_ranks_matches_reference(cid, synced_4):
    if _skip_reason(cid):
        pytest.skip(_skip_reason(cid))
    g = GOLDEN["class"][cid]
    if not _same(g["full"], g["merged"]):
        pytest.skip("reference merge is partition-dependent for this metric (window / ring)")
    for rank, res in enumerate(synced_4):
        assert not (isinstance(res[cid], dict) and "__raise__" in res[cid]), res[cid]
        assert_same(res[cid], g["full"], f"rank{rank}")


# metrics whose freshly constructed (never updated) state cannot be merged or computed in the
# reference either (window metrics with an unfilled window, Cat/AUC with empty inputs...) are
# skipped by the partition-invariance filter or by the reference raising on its own data
@pytest.mark.parametrize("cid", sorted(cases.CLASS))
def test_sync_with_an_empty_rank_matches_reference(cid, synced_3_with_empty_rank):
    """The reference's synclib has a dedicated protocol for ranks holding empty list states
    (synclib.py:73-102, 138-153); here rank 2 never calls update()."""
    if _skip_reason(cid):
        pytest.skip(_skip_reason(cid))
    g = GOLDEN["class"][cid]
    if not _same(g["full"], g["merged"]):
        pytest.skip("reference merge is partition-dependent for this metric (window / ring)")
    for rank, res in enumerate(synced_3_with_empty_rank):
        assert not (isinstance(res[cid], dict) and "__raise__" in res[cid]), res[cid]
        assert_same(res[cid], g["full"], f"rank{rank}")
