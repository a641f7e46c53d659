"""Direct RCCL communicator plumbing that needs no GPU (parallel/rccl_direct.py): the entry
points resolve from torch's librccl, the unique id is 128 bytes, the env switch and the
non-CUDA guard keep every other path on torch.distributed."""

import pytest
import torch

from torcheval_amd.ops import native, native_loaded
from torcheval_amd.parallel import rccl_direct

pytestmark = pytest.mark.skipif(not native_loaded(), reason="native extension not built")


def test_entry_points_resolve():
    assert native().rccl_available()


def test_unique_id_is_128_bytes_and_fresh():
    a = torch.zeros(128, dtype=torch.uint8)
    b = torch.zeros(128, dtype=torch.uint8)
    native().rccl_unique_id(a)
    native().rccl_unique_id(b)
    assert a.any() and not torch.equal(a, b)
    with pytest.raises(RuntimeError):
        native().rccl_unique_id(torch.zeros(64, dtype=torch.uint8))


def test_env_switch(monkeypatch):
    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "0")
    assert not rccl_direct.enabled()
    monkeypatch.setenv("TORCHEVAL_AMD_DIRECT_RCCL", "1")
    assert rccl_direct.enabled()


def test_cpu_tensors_never_get_a_communicator():
    assert rccl_direct.comm_for(None, 2, torch.device("cpu")) is None


def test_dispatcher_schemas_declare_mutation():
    ag = str(torch.ops.torcheval_amd.rccl_all_gather.default._schema)
    ar = str(torch.ops.torcheval_amd.rccl_all_reduce.default._schema)
    assert "Tensor(a!) dst" in ag and "Tensor(a!) t" in ar and "Tensor(b!)? out" in ar
