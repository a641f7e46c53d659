"""Runtime flags (torcheval_amd.config): trace ranges, validate, deterministic, disable_hip."""

import pytest
import torch
from torch.profiler import ProfilerActivity, profile

from torcheval_amd import config as cfg_mod
from torcheval_amd.config import config, flags
from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix


def test_flags_context_restores() -> None:
    before = (config.validate, config.deterministic, config.trace, config.disable_hip)
    with flags(validate=True, deterministic=True, trace=True, disable_hip=True):
        assert config.validate and config.deterministic and config.trace and config.disable_hip
    assert (config.validate, config.deterministic, config.trace, config.disable_hip) == before
    with pytest.raises(AttributeError):
        with flags(bogus=True):
            pass


def test_trace_ranges_in_profiler() -> None:
    m = MulticlassAccuracy()
    with flags(trace=True):
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            m.update(torch.rand(8, 3), torch.randint(0, 3, (8,)))
            m.compute()
    names = {e.name for e in prof.events()}
    assert "MulticlassAccuracy.update" in names and "MulticlassAccuracy.compute" in names
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        m.update(torch.rand(8, 3), torch.randint(0, 3, (8,)))
    assert "MulticlassAccuracy.update" not in {e.name for e in prof.events()}


def test_instrumented_once_and_subclass_safe() -> None:
    from torcheval_amd.metrics import BinaryAccuracy

    # inherited and overridden methods are wrapped exactly once
    assert getattr(BinaryAccuracy.update, "__tea_instrumented__", False)
    assert BinaryAccuracy.update.__wrapped__.__name__ == "update"
    assert not getattr(BinaryAccuracy.update.__wrapped__, "__tea_instrumented__", False)


def test_validate_flag_cpu_path_raises_immediately() -> None:
    m = MulticlassConfusionMatrix(3)
    with flags(validate=True):
        with pytest.raises(ValueError):
            m.update(torch.tensor([0, 1]), torch.tensor([0, 5]))


def test_trace_range_helper() -> None:
    with flags(trace=False):
        with cfg_mod.trace_range("x"):
            pass
    with flags(trace=True):
        with cfg_mod.trace_range("x"):
            pass
