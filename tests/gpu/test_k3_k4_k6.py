"""K3 (sort-scan AUROC/AUPRC), K4 (binned counts), K6 (NE sums) vs CPU fp64 references."""

import pytest
import torch

from torcheval_amd.metrics.functional import (
    binary_auprc,
    binary_auroc,
    binary_binned_auprc,
    binary_binned_auroc,
    binary_binned_precision_recall_curve,
    binary_normalized_entropy,
    multiclass_auprc,
    multiclass_auroc,
    multiclass_binned_auprc,
    multiclass_binned_auroc,
    multilabel_auprc,
    multilabel_binned_auprc,
)
from torcheval_amd.metrics.functional.classification._curve import binary_areas
from torcheval_amd.ops.binned import _binned_counts_aten, binned_counts

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _quantized(n, levels, g):
    # many ties, including groups that straddle the 4096-sample tiles of K3
    return (torch.randint(0, levels, (n,), generator=g).float() / levels)


@pytest.mark.parametrize("n", [1, 7, 4096, 4097, 50000, 1_000_003])
@pytest.mark.parametrize("levels", [0, 3, 1000])
def test_k3_binary_matches_cpu(n, levels):
    g = torch.Generator().manual_seed(n + levels)
    x = torch.rand(n, generator=g) if levels == 0 else _quantized(n, levels, g)
    t = torch.randint(0, 2, (n,), generator=g)
    roc_c, pr_c = binary_areas(x, t, None, roc=True, pr=True)
    roc_g, pr_g = binary_areas(x.to(DEV), t.to(DEV), None, roc=True, pr=True)
    torch.testing.assert_close(roc_g.cpu(), roc_c, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(pr_g.cpu(), pr_c, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("weighted", [False, True])
def test_k3_tie_groups_at_the_window_edges(weighted):
    """Tie groups of every length around the 64-sample window that resolves a group straddling a
    1024-sample tile edge (1-3, 62-66, 127-129, 1000+): the window path, its fallback to the
    binary search, and groups spanning whole tiles, against the CPU fp64 reference."""
    g = torch.Generator().manual_seed(17 + weighted)
    sizes = torch.tensor([1, 2, 3, 62, 63, 64, 65, 66, 127, 128, 129, 1500])
    reps = sizes[torch.randint(0, len(sizes), (2500,), generator=g)]
    vals = torch.randperm(len(reps), generator=g).float() / len(reps)
    x = torch.repeat_interleave(vals, reps)
    x = x[torch.randperm(len(x), generator=g)]
    n = len(x)
    t = torch.randint(0, 2, (n,), generator=g)
    w = torch.rand(n, generator=g) if weighted else None
    roc_c, pr_c = binary_areas(x, t, w, roc=True, pr=True)
    roc_g, pr_g = binary_areas(x.to(DEV), t.to(DEV), None if w is None else w.to(DEV), roc=True, pr=True)
    torch.testing.assert_close(roc_g.cpu(), roc_c, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(pr_g.cpu(), pr_c, rtol=1e-9, atol=1e-12)


def test_k3_all_equal_scores_and_degenerate():
    for x, t in [
        (torch.full((20000,), 0.5), torch.randint(0, 2, (20000,))),
        (torch.rand(9000), torch.zeros(9000, dtype=torch.long)),
        (torch.rand(9000), torch.ones(9000, dtype=torch.long)),
    ]:
        roc_c, pr_c = binary_areas(x, t, None, roc=True, pr=True)
        roc_g, pr_g = binary_areas(x.to(DEV), t.to(DEV), None, roc=True, pr=True)
        torch.testing.assert_close(roc_g.cpu(), roc_c)
        torch.testing.assert_close(pr_g.cpu(), pr_c)


def test_k3_weighted_multitask_and_dtypes():
    g = torch.Generator().manual_seed(3)
    x = _quantized(3 * 30000, 50, g).view(3, 30000)
    t = torch.randint(0, 2, (3, 30000), generator=g).float()
    w = torch.rand(3, 30000, generator=g)
    exp = binary_auroc(x, t, num_tasks=3, weight=w)
    got = binary_auroc(x.to(DEV), t.to(DEV), num_tasks=3, weight=w.to(DEV))
    torch.testing.assert_close(got.cpu(), exp, rtol=1e-9, atol=1e-12)
    assert got.dtype == torch.float64
    xd = x.double()
    torch.testing.assert_close(binary_auroc(xd[0].to(DEV), t[0].to(DEV)).cpu(), binary_auroc(xd[0], t[0]))
    xb = x.bfloat16()
    torch.testing.assert_close(binary_auprc(xb[1].to(DEV), t[1].to(DEV)).cpu(), binary_auprc(xb[1], t[1]))


@pytest.mark.parametrize("C", [2, 10, 130])
def test_k3_multiclass_multilabel(C):
    g = torch.Generator().manual_seed(C)
    X = _quantized(20000 * C, 97, g).view(20000, C)
    y = torch.randint(0, C, (20000,), generator=g)
    torch.testing.assert_close(
        multiclass_auroc(X.to(DEV), y.to(DEV), num_classes=C, average=None).cpu(),
        multiclass_auroc(X, y, num_classes=C, average=None),
    )
    torch.testing.assert_close(
        multiclass_auprc(X.to(DEV), y.to(DEV), average=None).cpu(), multiclass_auprc(X, y, average=None)
    )
    if C >= 2:
        Y = torch.randint(0, 2, (20000, C), generator=g)
        torch.testing.assert_close(
            multilabel_auprc(X.to(DEV), Y.to(DEV), average=None).cpu(), multilabel_auprc(X, Y, average=None)
        )


@pytest.mark.parametrize("T", [1, 5, 100, 200, 1000])
@pytest.mark.parametrize("mode", [0, 1])
def test_k4_binned_counts(T, mode):
    g = torch.Generator().manual_seed(T * 7 + mode)
    C = 37
    x = torch.rand(5003, C, generator=g)
    x[:50] = 0.0
    x[50:100] = 1.0
    thr = torch.cat([torch.tensor([0.0, 1.0]), torch.rand(max(T - 2, 0), generator=g)]).sort().values[:T]
    t = torch.randint(0, C, (5003,), generator=g) if mode == 1 else torch.randint(0, 2, (5003, C), generator=g)
    exp = _binned_counts_aten(x, t, thr, mode)
    got = binned_counts(x.to(DEV), t.to(DEV), thr.to(DEV), mode)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a.cpu(), b)
    # strided (task-major) view, as used by multi-task binned metrics
    xt = x.t().contiguous()
    got2 = binned_counts(xt.to(DEV).t(), t.to(DEV), thr.to(DEV), mode)
    for a, b in zip(got2, exp):
        torch.testing.assert_close(a.cpu(), b)


@pytest.mark.parametrize("case", ["uniform_f32", "bf16_bool", "float_target", "edge_values", "slabs"])
def test_k4_dense_path(case):
    """[T+1] x C histograms that fit one block's LDS take the dense path (packed 16-bit
    counters, slab flush + reduce); rows beyond 512 x 65535 elements split into row slabs."""
    g = torch.Generator().manual_seed(hash(case) % 1000)
    n, C, T, mode = 20000, 50, 101, 1
    if case == "slabs":
        n, C = 700_000, 50  # 35M elements -> 2 row slabs
    x = torch.rand(n, C, generator=g)
    thr = torch.linspace(0, 1, T)
    if case == "edge_values":
        x[:100] = float("nan")
        x[100:200] = -0.5
        x[200:300] = 1.5
        x[300:400] = thr[37]  # exactly on a threshold
        thr = torch.cat([torch.tensor([0.0]), torch.rand(T - 2, generator=g).sort().values, torch.tensor([1.0])])
    t = torch.randint(0, C, (n,), generator=g)
    if case in ("bf16_bool", "float_target"):
        mode = 0
        t = torch.randint(0, 2, (n, C), generator=g)
        if case == "bf16_bool":
            x = x.bfloat16()
            t = t.bool()
        else:
            t = t.float()
    exp = _binned_counts_aten(x.float() if x.dtype == torch.bfloat16 else x, t.long() if t.dtype == torch.bool else t,
                              thr, mode)
    got = binned_counts(x.to(DEV), t.to(DEV), thr.to(DEV), mode)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a.cpu(), b)


@pytest.mark.parametrize("shape", [(3000, 1000, 100), (2000, 100, 1000), (500, 7, 8000), (4000, 300, 57)])
@pytest.mark.parametrize("mode", [0, 1])
def test_k4_dense_class_chunks(shape, mode):
    """[T+1] x C beyond one block's LDS: the dense path splits classes into chunks (grid.y),
    including a ragged last chunk and column-major (transposed) scores."""
    n, C, T = shape
    g = torch.Generator().manual_seed(n + C + T)
    x = torch.rand(C, n, generator=g).t() if C == 300 else torch.rand(n, C, generator=g)
    thr = torch.linspace(0, 1, T)
    t = torch.randint(0, C, (n,), generator=g) if mode == 1 else torch.randint(0, 2, (n, C), generator=g)
    exp = _binned_counts_aten(x.contiguous(), t, thr, mode)
    got = binned_counts(x.to(DEV), t.to(DEV), thr.to(DEV), mode)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a.cpu(), b)


@pytest.mark.parametrize("T", [2, 3, 100, 201, 2000])
@pytest.mark.parametrize("mode", [0, 1])
def test_k4_uniform_threshold_boundaries(T, mode):
    """Int thresholds are the cached linspace: the kernels bin arithmetically and only verify
    near a threshold.  Feed exact thresholds, their float neighbours and out-of-range / NaN
    values, for both the dense and the (binary, small-T) sparse kernels."""
    from torcheval_amd.metrics.functional.tensor_utils import _create_threshold_tensor

    thr = _create_threshold_tensor(T, torch.device(DEV))
    tc = thr.cpu()
    vals = torch.cat([tc, torch.nextafter(tc, torch.tensor(2.0)), torch.nextafter(tc, torch.tensor(-1.0)),
                      torch.tensor([0.0, 1.0, -0.0, -1e-30, 1e-30, 1.5, -3.0, float("nan"), float("inf")])])
    g = torch.Generator().manual_seed(T + mode)
    for C in (1, 3, 64):
        n = vals.numel() * 4
        x = vals[torch.randint(0, vals.numel(), (n, C), generator=g)]
        t = torch.randint(0, C, (n,), generator=g) if mode == 1 else torch.randint(0, 2, (n, C), generator=g)
        if mode == 1 and C == 1:
            continue
        exp = _binned_counts_aten(x, t, tc, mode)
        got = binned_counts(x.to(DEV), t.to(DEV), thr, mode)
        for a, b in zip(got, exp):
            torch.testing.assert_close(a.cpu(), b)


def test_binned_metrics_gpu_vs_cpu():
    g = torch.Generator().manual_seed(11)
    x = torch.rand(4, 3000, generator=g)
    t = torch.randint(0, 2, (4, 3000), generator=g)
    for fn, kw in [(binary_binned_auroc, dict(num_tasks=4, threshold=50)),
                   (binary_binned_auprc, dict(num_tasks=4, threshold=50))]:
        a, _ = fn(x.to(DEV), t.to(DEV), **kw)
        b, _ = fn(x, t, **kw)
        torch.testing.assert_close(a.cpu(), b)
    p1 = binary_binned_precision_recall_curve(x[0].to(DEV), t[0].to(DEV), threshold=10)
    p2 = binary_binned_precision_recall_curve(x[0], t[0], threshold=10)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a.cpu(), b)
    X = torch.rand(3000, 6, generator=g)
    y = torch.randint(0, 6, (3000,), generator=g)
    torch.testing.assert_close(multiclass_binned_auroc(X.to(DEV), y.to(DEV), num_classes=6)[0].cpu(),
                               multiclass_binned_auroc(X, y, num_classes=6)[0])
    torch.testing.assert_close(multiclass_binned_auroc(X.to(DEV), y.to(DEV), num_classes=6, one_vs_rest=True)[0].cpu(),
                               multiclass_binned_auroc(X, y, num_classes=6, one_vs_rest=True)[0])
    torch.testing.assert_close(multiclass_binned_auprc(X.to(DEV), y.to(DEV))[0].cpu(), multiclass_binned_auprc(X, y)[0])
    Y = torch.randint(0, 2, (3000, 6), generator=g)
    torch.testing.assert_close(multilabel_binned_auprc(X.to(DEV), Y.to(DEV))[0].cpu(), multilabel_binned_auprc(X, Y)[0])


@pytest.mark.parametrize("from_logits", [False, True])
def test_k6_normalized_entropy(from_logits):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 20000, generator=g) if from_logits else torch.rand(3, 20000, generator=g)
    x[0, :10] = 0.0 if not from_logits else -50.0
    t = torch.randint(0, 2, (3, 20000), generator=g).float()
    w = torch.rand(3, 20000, generator=g)
    exp = binary_normalized_entropy(x, t, weight=w, num_tasks=3, from_logits=from_logits)
    got = binary_normalized_entropy(x.to(DEV), t.to(DEV), weight=w.to(DEV), num_tasks=3, from_logits=from_logits)
    torch.testing.assert_close(got.cpu(), exp, rtol=1e-6, atol=1e-9)


def test_k6_range_error():
    with pytest.raises(ValueError, match="should be probability in range"):
        binary_normalized_entropy(torch.tensor([0.2, 1.5]).to(DEV), torch.tensor([0.0, 1.0]).to(DEV))


# ----------------------------------------------------------------------------- K3a radix sort
@pytest.mark.parametrize("rows,n", [(1, 1), (1, 4095), (1, 4096), (1, 4097), (1, 1_000_003), (7, 9000), (100, 1000)])
@pytest.mark.parametrize("levels", [0, 5])
def test_k3a_radix_sort_matches_torch(rows, n, levels):
    from torcheval_amd.ops import native

    g = torch.Generator().manual_seed(rows * 1000 + n + levels)
    x = torch.randn(rows, n, generator=g) if levels == 0 else torch.randint(0, levels, (rows, n), generator=g).float() - 2
    if n > 10:
        x[0, 3] = float("nan")
        x[0, 5] = -0.0
        x[0, 6] = 0.0
        x[0, 7] = float("inf")
        x[0, 8] = float("-inf")
    xd = x.to(DEV)
    s = torch.empty_like(xd)
    idx = torch.empty(xd.shape, dtype=torch.int32, device=DEV)
    native().sort_desc(xd, s, idx)
    ref = torch.sort(x, dim=-1, descending=True).values
    torch.testing.assert_close(s.cpu(), ref, equal_nan=True, rtol=0, atol=0)
    # permutation: gathers the sorted values and is a bijection per row
    g_back = torch.gather(x, 1, idx.cpu().long())
    torch.testing.assert_close(g_back, ref, equal_nan=True, rtol=0, atol=0)
    assert torch.equal(idx.cpu().long().sort(dim=1).values, torch.arange(n).expand(rows, n))
    if levels:
        # stability: LSD radix is stable, equal keys keep ascending source order
        ii = idx.cpu().long()
        same = s.cpu()[:, 1:] == s.cpu()[:, :-1]
        assert bool((ii[:, 1:] > ii[:, :-1])[same].all())


def test_k3a_strided_rows():
    from torcheval_amd.ops import native

    big = torch.rand(4, 5000, device=DEV)
    x = big[:, :4500]
    s = torch.empty(4, 4500, device=DEV)
    idx = torch.empty(4, 4500, dtype=torch.int32, device=DEV)
    native().sort_desc(x, s, idx)
    torch.testing.assert_close(s, torch.sort(x, dim=-1, descending=True).values, rtol=0, atol=0)


@pytest.mark.parametrize("n,c", [(1, 1), (63, 65), (100_000, 100), (4097, 3), (4100, 68), (8, 4), (132, 256)])
@pytest.mark.parametrize("strided", [False, True])
def test_tiled_transpose(n, c, strided):
    # (n, c multiples of 4 with aligned rows take the 16-B kernel, ragged tiles included)
    from torcheval_amd.ops import native

    x = torch.randn(n, c + 8, device=DEV)[:, :c] if strided else torch.randn(n, c, device=DEV)
    out = torch.empty(c, n, device=DEV)
    native().transpose_f32(x, out)
    assert torch.equal(out, x.t().contiguous())


@pytest.mark.parametrize("n,levels,weighted", [(5000, 0, False), (70_000, 37, True), (3000, 3, False)])
def test_k3_shard_offsets_match_cpu(n, levels, weighted):
    """K3 with (TP0, FP0) shard offsets + raw sums (the sample-sharded AUROC path) vs ATen."""
    from torcheval_amd.metrics.functional.classification._curve import raw_area_sums

    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, generator=g)
    if levels:
        x = (x * levels).floor() / levels
    t = torch.randint(0, 2, (n,), generator=g)
    w = torch.rand(n, generator=g, dtype=torch.float64) if weighted else None
    for tp0, fp0 in [(0.0, 0.0), (123.0, 456.5)]:
        want = raw_area_sums(x, t.float(), w, tp0, fp0)
        got = raw_area_sums(x.cuda(), t.float().cuda(), None if w is None else w.cuda(), tp0, fp0)
        torch.testing.assert_close(got.cpu(), want, rtol=1e-9, atol=1e-6)
