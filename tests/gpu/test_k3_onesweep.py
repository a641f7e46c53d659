"""K3a onesweep sort (csrc/kernels/radix.hip: one histogram launch + four look-back passes):
exact agreement with torch.sort over a sequence of sorts whose shapes change from call to call
(the self-cleaning status / group planes and digit totals must never leak a stale flag into the
next shape), with payloads, ties, NaN / +-0 / +-inf, and shapes past the onesweep tiling limit
(the legacy upsweep / downsweep path) interleaved."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(x: torch.Tensor, payload=None, kind: int = 0) -> None:
    from torcheval_amd.ops import native

    xd = x.to(DEV)
    s = torch.empty_like(xd)
    idx = torch.empty(xd.shape, dtype=torch.int32, device=DEV)
    native().sort_desc(xd, s, idx, None if payload is None else payload.to(DEV), kind)
    ref_vals, ref_idx = torch.sort(x, dim=-1, descending=True, stable=True)
    torch.testing.assert_close(s.cpu(), ref_vals, equal_nan=True, rtol=0, atol=0)
    got = idx.cpu().long()
    if kind == 0:
        # the LSD sort is stable: equal keys keep ascending source order (== torch's stable sort,
        # NaN included; -0 / +0 compare equal for both)
        assert torch.equal(got, ref_idx), "permutation differs from the stable reference"
    elif kind == 1:
        want = torch.gather(payload.float().expand(x.shape) if payload.dim() == 1 else payload.float(), 1, ref_idx)
        torch.testing.assert_close(idx.cpu().view(torch.float32), want, rtol=0, atol=0)
    else:
        want = torch.gather(payload.long().expand(x.shape) if payload.dim() == 1 else payload.long(), 1, ref_idx)
        assert torch.equal(got, want)


def _keys(rows: int, n: int, seed: int, levels: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(rows, n, generator=g) if levels == 0 else torch.randint(0, levels, (rows, n), generator=g).float() / levels
    if n > 12:
        x[0, 3] = float("nan")
        x[0, 5] = -0.0
        x[0, 6] = 0.0
        x[0, 7] = float("inf")
        x[0, 8] = float("-inf")
        x[-1, n - 1] = float("nan")
    return x


def test_shape_sequence_keeps_the_workspace_clean():
    g = torch.Generator().manual_seed(5)
    # (1, 2_097_152) is exactly 1024 tiles (the onesweep limit), one key more takes the legacy
    # sort; (8, 500_000) crosses to 16-round tiles; 9 and 100 rows take the legacy sort
    shapes = [(1, 1_000_000), (1, 3), (3, 70_000), (1, 2_100_000), (1, 4096), (100, 1000), (1, 1_000_000),
              (2, 5_000_000 // 2 + 17), (1, 2049), (8, 131_072), (1, 999_999), (1, 1), (1, 2_097_152),
              (1, 2_097_153), (8, 500_000), (9, 50_000)]
    from torcheval_amd.ops import native

    for step, (rows, n) in enumerate(shapes * 2):
        levels = int(torch.randint(0, 3, (1,), generator=g)) * 7
        _check(_keys(rows, n, 100 + step, levels))
    # no look-back spin of any of these sorts hit its bound
    assert native().sort_desc_timeouts(torch.empty(1, device=DEV)) == 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.int64, torch.uint8, torch.bool])
def test_target_payload(dtype):
    x = _keys(1, 700_001, 7, 0)
    t = (torch.rand(700_001) < 0.3)
    t = t.to(dtype) if dtype != torch.float32 else t.float() * 0.75
    _check(x, t, 1)


def test_label_payload_shared_by_rows():
    x = _keys(5, 80_000, 9, 11)
    lab = torch.randint(0, 100, (80_000,))
    _check(x, lab, 2)
    _check(x, lab.int(), 2)


def test_binary_auroc_1m_matches_cpu_across_repeats():
    from torcheval_amd.metrics.functional import binary_auprc, binary_auroc

    g = torch.Generator().manual_seed(3)
    for rep in range(3):
        x = torch.rand(1_000_000, generator=g)
        x[:1000] = 0.5  # a long tie group straddling tiles
        t = (torch.rand(1_000_000, generator=g) < 0.4).long()
        want_roc = binary_auroc(x.double(), t)
        want_pr = binary_auprc(x.double(), t)
        torch.testing.assert_close(binary_auroc(x.to(DEV), t.to(DEV)).cpu().double(), want_roc.double(), rtol=1e-9, atol=1e-12)
        torch.testing.assert_close(binary_auprc(x.to(DEV), t.to(DEV)).cpu().double(), want_pr.double(), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("group_len,offset", [(40, 1000), (64, 990), (100, 1000), (1100, 1000), (3000, 500),
                                              (2048, 1024), (70, 1023), (63, 961), (5000, 0)])
def test_tie_groups_across_tiles(group_len, offset):
    """Long tie groups straddling 1024-sample tiles at every offset class (short groups resolved
    from the edge window, long ones by the binary search), weighted and unweighted, one and
    three rows, against the CPU oracle."""
    from torcheval_amd.metrics.functional import binary_auprc, binary_auroc

    g = torch.Generator().manual_seed(group_len + offset)
    n = 20_000
    x = torch.rand(n, generator=g)
    order = torch.argsort(x, descending=True)
    x[order[offset:offset + group_len]] = float(x[order[offset]])  # one group starting at `offset` in sorted order
    x[order[7000:7000 + group_len // 2 + 1]] = float(x[order[7000]])
    t = (torch.rand(n, generator=g) < 0.5).long()
    w = torch.rand(n, generator=g).double()
    for weight in (None, w):
        kw = {} if weight is None else {"weight": weight}
        want = binary_auroc(x.double(), t, **kw)
        got = binary_auroc(x.to(DEV), t.to(DEV), **({} if weight is None else {"weight": weight.to(DEV)}))
        torch.testing.assert_close(got.cpu().double(), want.double(), rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(binary_auprc(x.to(DEV), t.to(DEV)).cpu().double(), binary_auprc(x.double(), t).double(),
                               rtol=1e-6, atol=1e-9)
    # several rows (num_tasks): the per-row tags / prefixes
    xs = torch.stack([x, x.flip(0), torch.rand(n, generator=g)])
    ts = torch.stack([t, t, t.flip(0)])
    torch.testing.assert_close(binary_auroc(xs.to(DEV), ts.to(DEV), num_tasks=3).cpu().double(),
                               binary_auroc(xs.double(), ts, num_tasks=3).double(), rtol=1e-9, atol=1e-12)


def _tile_sums_cpu(sorted_payload: torch.Tensor, kind: int) -> torch.Tensor:
    """(sum t, sum 1 - t) per 1024-sample tile of each row, float64, from the sorted payload."""
    rows, n = sorted_payload.shape
    if kind == 1:
        t = sorted_payload.view(torch.float32).double()
    else:
        t = (sorted_payload.long() == torch.arange(rows)[:, None]).double()
    b = (1.0 - t.float()).double()
    tiles = (n + 1023) // 1024
    pad = tiles * 1024 - n
    t = torch.nn.functional.pad(t, (0, pad)).view(rows, tiles, 1024).sum(-1)
    b = torch.nn.functional.pad(b, (0, pad)).view(rows, tiles, 1024).sum(-1)
    return torch.stack([t, b], -1)


@pytest.mark.parametrize("rows,n,kind,frac", [(1, 1_000_000, 1, False), (1, 1, 1, False), (1, 1025, 1, False),
                                              (3, 70_001, 1, False), (8, 20_000, 2, False), (2, 2_100_000, 1, False),
                                              (1, 300_000, 1, True), (5, 4097, 2, False)])
def test_tile_sum_fold_matches_the_sorted_payload(rows, n, kind, frac):
    """The last onesweep pass's tile-sum fold (sort_desc(fold=...)) against the tile totals of its
    own sorted payload; then auc_scan with the fold equals auc_scan without it."""
    import os

    from torcheval_amd.ops import native

    if os.environ.get("TORCHEVAL_AMD_K3_ONESWEEP") == "0":
        pytest.skip("the fold rides the onesweep sort, turned off in this process")

    g = torch.Generator().manual_seed(rows * 7 + n)
    x = _keys(rows, n, n, 5 if n > 1000 else 0)
    if kind == 1:
        pl = torch.rand(rows, n, generator=g) if frac else (torch.rand(rows, n, generator=g) < 0.4).float()
    else:
        pl = torch.randint(0, rows + 2, (n,), generator=g)
    xd = x.to(DEV)
    s = torch.empty_like(xd)
    idx = torch.empty(xd.shape, dtype=torch.int32, device=DEV)
    fold = torch.full((rows, (n + 1023) // 1024, 2), float("nan"), dtype=torch.float64, device=DEV)
    assert native().sort_desc(xd, s, idx, pl.to(DEV), kind, fold), "onesweep path expected to fold"
    want = _tile_sums_cpu(idx.cpu(), kind)
    if frac:
        torch.testing.assert_close(fold.cpu(), want, rtol=1e-12, atol=1e-9)
    else:
        assert torch.equal(fold.cpu(), want)
    # the scan with and without the fold
    out = [torch.empty(rows, dtype=torch.float64, device=DEV) for _ in range(4)]
    tgt = pl.to(DEV)
    native().auc_scan(s, idx, tgt, None, kind == 2, out[0], out[1], None, None, kind)
    native().auc_scan(s, idx, tgt, None, kind == 2, out[2], out[3], None, None, kind, fold)
    torch.testing.assert_close(out[2], out[0], rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(out[3], out[1], rtol=1e-12, atol=1e-12)


def test_fold_not_taken_off_the_onesweep_path():
    """Past the onesweep tiling (or without a payload) the sort reports no fold."""
    from torcheval_amd.ops import native

    x = torch.rand(9, 5000, device=DEV)
    s = torch.empty_like(x)
    idx = torch.empty(x.shape, dtype=torch.int32, device=DEV)
    fold = torch.empty(9, 5, 2, dtype=torch.float64, device=DEV)
    assert not native().sort_desc(x, s, idx, torch.zeros(9, 5000, device=DEV), 1, fold)
    x1 = torch.rand(1, 5000, device=DEV)
    s1, i1 = torch.empty_like(x1), torch.empty(x1.shape, dtype=torch.int32, device=DEV)
    assert not native().sort_desc(x1, s1, i1, None, 0, torch.empty(1, 5, 2, dtype=torch.float64, device=DEV))
