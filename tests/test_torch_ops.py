"""The native kernels are registered with the torch dispatcher (torch.ops.torcheval_amd.*):
CPU (host twin) and Meta kernels here; the CUDA kernels in tests/gpu/test_torch_ops_gpu.py."""

import pytest
import torch

from torcheval_amd.ops import native_loaded

pytestmark = pytest.mark.skipif(not native_loaded(), reason="native extension not built")


def test_row_sums_cpu_through_dispatcher():
    x, t = torch.rand(4, 50), torch.rand(4, 50)
    outs = [torch.zeros(4, dtype=torch.float64), torch.full((4,), 1.0)]
    codes = [0 * 8 + 1, 3 * 8 + 1]  # WX add, SSE add
    torch.ops.torcheval_amd.row_sums(x, t, None, 2.0, outs, codes, 4)
    torch.testing.assert_close(outs[0], 2.0 * x.double().sum(1))
    torch.testing.assert_close(outs[1], 1.0 + ((x - t) ** 2).sum(1), rtol=1e-5, atol=1e-5)


def test_meta_kernels_accept_shapes():
    x = torch.empty(4, 50, device="meta")
    out = torch.empty(4, dtype=torch.float64, device="meta")
    torch.ops.torcheval_amd.row_sums(x, None, None, 1.0, [out], [1], 4)
    s = torch.empty(2, 10, device="meta")
    o = torch.empty(2, 10, dtype=torch.int32, device="meta")
    torch.ops.torcheval_amd.sort_desc(s, s, o, None, 0)


def test_schemas_declare_mutation():
    schema = str(torch.ops.torcheval_amd.rafp.default._schema)
    assert "Tensor(a!) out_max_recall" in schema and "Tensor(b!) out_best_thr" in schema
    assert "Tensor(a!)[] outs" in str(torch.ops.torcheval_amd.row_sums.default._schema)
