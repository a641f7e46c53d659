"""Staged FID updates (fid.py: activations staged in HBM, K8 once per full stage or on read).

Staging is on the native path only; here it is forced on the CPU (``_stageable``) with a
small stage so the flush-on-read property logic runs against the unstaged metric.
"""
import copy
import os
import pickle

import pytest
import torch

from torcheval_amd.metrics.image import fid as fid_mod
from torcheval_amd.metrics.image.fid import FrechetInceptionDistance
from torcheval_amd.utils.test_utils.dist_pool import run_distributed

D = 8
CAP = 16
STATES = ("real_sum", "real_cov_sum", "fake_sum", "fake_cov_sum", "num_real_images", "num_fake_images")


def _force_staging(cap: int = CAP) -> None:
    os.environ["TORCHEVAL_AMD_FID_STAGE_ROWS"] = str(cap)
    fid_mod._stageable = lambda act: True


@pytest.fixture
def staged(monkeypatch):
    monkeypatch.setenv("TORCHEVAL_AMD_FID_STAGE_ROWS", str(CAP))
    monkeypatch.setattr(fid_mod, "_stageable", lambda act: True)


def _metric() -> FrechetInceptionDistance:
    return FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=D)


def _feed(m, seed: int, sizes=(3, 7, 5, 9, 20, 1)):
    g = torch.Generator().manual_seed(seed)
    for i, b in enumerate(sizes):
        m.update_activations(torch.rand(b, D, generator=g) + (0.3 if i % 2 else 0.0), is_real=i % 3 != 1)
    return m


def _plain(seed: int, sizes=(3, 7, 5, 9, 20, 1)):
    old = fid_mod._stageable
    fid_mod._stageable = lambda act: False
    try:
        return _feed(_metric(), seed, sizes)
    finally:
        fid_mod._stageable = old


def _assert_states(a, b) -> None:
    for name in STATES:
        torch.testing.assert_close(getattr(a, name), getattr(b, name), rtol=1e-5, atol=1e-5)


def test_staged_matches_unstaged(staged):
    m = _feed(_metric(), 0)
    assert sum(m._stage_rows) > 0  # something is still staged before the read
    ref = _plain(0)
    torch.testing.assert_close(m.compute(), ref.compute(), rtol=1e-4, atol=1e-4)
    _assert_states(m, ref)
    assert m._stage_rows == [0, 0]


def test_count_read_flushes(staged):
    m = _metric()
    m.update_activations(torch.rand(4, D), is_real=True)
    assert m._stage_rows == [4, 0]
    assert int(m.num_real_images) == 4
    assert m._stage_rows == [0, 0]


def test_state_dict_and_load(staged):
    m = _feed(_metric(), 1)
    sd = m.state_dict()
    ref = _plain(1)
    for name in STATES:
        torch.testing.assert_close(sd[name], getattr(ref, name), rtol=1e-5, atol=1e-5)
    n = _metric()
    n.update_activations(torch.rand(5, D), is_real=True)  # staged rows belong to the old value
    n.load_state_dict(sd)
    _assert_states(n, ref)


def test_reset_discards_staged(staged):
    m = _metric()
    m.update_activations(torch.rand(5, D), is_real=True)
    m.update_activations(torch.rand(3, D), is_real=False)
    m.reset()
    assert int(m.num_real_images) == 0 and int(m.num_fake_images) == 0
    assert float(m.real_cov_sum.abs().sum()) == 0.0
    _feed(m, 2)
    _assert_states(m, _plain(2))


def test_copies_carry_staged_rows(staged):
    m = _metric()
    m.update_activations(torch.rand(6, D), is_real=True)
    for c in (copy.deepcopy(m), pickle.loads(pickle.dumps(m)), copy.copy(m)):
        assert int(c.num_real_images) == 6
        assert c._stage == [None, None]
    assert int(m.num_real_images) == 6


def test_merge_state(staged):
    a = _feed(_metric(), 3)
    b = _feed(_metric(), 4, sizes=(11, 2, 6))
    a.merge_state([b])
    ra, rb = _plain(3), _plain(4, sizes=(11, 2, 6))
    ra.merge_state([rb])
    _assert_states(a, ra)


def test_oversized_batch_bypasses_stage(staged):
    m = _metric()
    m.update_activations(torch.rand(3, D), is_real=True)
    m.update_activations(torch.rand(CAP + 5, D), is_real=True)  # > stage: direct K8 path
    assert int(m.num_real_images) == CAP + 8


def _sync_job(rank: int, world_size: int):
    _force_staging()
    from torcheval_amd.metrics.toolkit import sync_and_compute

    m = _feed(_metric(), 10 + rank, sizes=(4, 3, 9, 2, 5 + rank))
    return float(sync_and_compute(m)), m._stage_rows


def test_sync_and_compute_gloo():
    ra, rb = _plain(10, sizes=(4, 3, 9, 2, 5)), _plain(11, sizes=(4, 3, 9, 2, 6))
    ra.merge_state([rb])
    want = float(ra.compute())
    for got, _ in run_distributed(_sync_job, 2):
        assert got == pytest.approx(want, rel=1e-4, abs=1e-4)
