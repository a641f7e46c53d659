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


HOT_OPS = ("micro_accuracy", "cls_counts", "binary_counts", "rank_scores", "multilabel_counts", "binned_counts",
           "binned_finalize", "auc_scan", "sort_desc", "rafp", "curve_count", "curve_emit", "merge_sorted_runs",
           "retrieval_topk_update", "row_sums", "column_moments", "ne_sums", "perplexity_sums", "fid_cov_update",
           "sym_eigvals", "potrf_block", "cholesky_factor", "pivchol", "cov_finalize", "sym_fill_upper", "fid_finish", "trapz_sorted", "transpose_f32", "seg_reduce_rows")


@pytest.mark.parametrize("name", HOT_OPS)
def test_every_native_entry_point_is_a_dispatcher_op(name):
    op = getattr(torch.ops.torcheval_amd, name).default
    schema = op._schema
    # every kernel that writes into caller tensors says so in its schema
    returns_only = name in ("merge_sorted_runs",)
    assert returns_only or any(a.alias_info is not None and a.alias_info.is_write for a in schema.arguments) \
        or len(schema.returns) > 0, str(schema)


def test_meta_kernels_of_update_ops():
    m = "meta"
    x = torch.empty(64, 100, device=m)
    y = torch.empty(64, dtype=torch.int64, device=m)
    c, t = torch.empty((), device=m), torch.empty((), device=m)
    torch.ops.torcheval_amd.micro_accuracy(x, y, c, t)
    cm = torch.empty(100 * 100, device=m)
    torch.ops.torcheval_amd.cls_counts(x, y, 1, 100, None, None, None, None, None, cm, None)
    thr = torch.empty(50, device=m)
    tp, fp, fn = (torch.empty(50, 100, device=m) for _ in range(3))
    torch.ops.torcheval_amd.binned_counts(x, y, thr, 1, tp, fp, fn, 0)
    assert torch.ops.torcheval_amd.rank_scores(x, y, 0, 5, None).shape == (64,)
    rows, out = torch.empty(64, dtype=torch.uint8, device=m), torch.empty(32, dtype=torch.uint8, device=m)
    torch.ops.torcheval_amd.seg_reduce_rows(rows, out, 2, [0], [8], [0], [0])
