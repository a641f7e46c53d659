"""K3m (csrc/kernels/merge.hip): merge-path merge of descending runs on the GPU, and the
sorted-run AUROC / AUPRC compute it feeds, against a stable sort / the union compute."""

import pytest
import torch

from torcheval_amd.metrics.functional import binary_auprc, binary_auroc
from torcheval_amd.metrics.functional.classification._curve import merged_areas, sort_run
from torcheval_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _runs(sizes, levels, seed, nan=False):
    g = torch.Generator().manual_seed(seed)
    out = []
    for n in sizes:
        x = torch.randint(0, levels, (n,), generator=g).float() / levels
        if nan and n > 3:
            x[n // 2] = float("nan")
        out.append(torch.sort(x, descending=True, stable=True).values)
    return out


@pytest.mark.parametrize("sizes,levels", [((5, 0, 7), 3), ((1,), 5), ((1000, 999, 1, 2048, 2049), 17),
                                          ((1_000_000, 500_001, 3), 1 << 30), ((250_000,) * 8, 1000)])
def test_merge_matches_stable_sort(sizes, levels):
    runs = _runs(sizes, levels, sum(sizes), nan=True)
    x = torch.cat(runs)
    s, o = native().merge_sorted_runs([r.to(DEV) for r in runs])
    s_cpu, o_cpu = native().merge_sorted_runs(runs)
    torch.testing.assert_close(s.cpu(), s_cpu, equal_nan=True, rtol=0, atol=0)
    assert torch.equal(o.cpu(), o_cpu)  # same stable order as the host merge
    want, perm = torch.sort(x, descending=True, stable=True)
    torch.testing.assert_close(s.cpu(), want, equal_nan=True, rtol=0, atol=0)
    assert torch.equal(o.cpu().long(), perm)  # positions = the stable permutation
    # a carried payload comes out in the same order
    pays = [torch.arange(r.numel(), dtype=torch.int32) * 3 + i for i, r in enumerate(runs)]
    _, p = native().merge_sorted_runs([r.to(DEV) for r in runs], [q.to(DEV) for q in pays])
    assert torch.equal(p.cpu(), torch.cat(pays)[perm])


@pytest.mark.parametrize("R,n", [(2, 100_000), (8, 125_000), (3, 7)])
def test_merged_areas_match_union(R, n):
    g = torch.Generator().manual_seed(R * n)
    xs = [(torch.randint(0, 5000, (n,), generator=g) / 5000.0).to(DEV) for _ in range(R)]
    ts = [torch.randint(0, 2, (n,), generator=g).to(DEV) for _ in range(R)]
    ws = [torch.rand(n, generator=g, dtype=torch.float64).to(DEV) for _ in range(R)]
    runs = [sort_run(x, t, w) for x, t, w in zip(xs, ts, ws)]
    roc, pr = merged_areas([r[0] for r in runs], [r[1] for r in runs], None, roc=True, pr=True)
    X, T, W = torch.cat(xs), torch.cat(ts), torch.cat(ws)
    torch.testing.assert_close(roc[0], binary_auroc(X, T).double(), rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(pr[0].float(), binary_auprc(X, T), rtol=1e-6, atol=1e-6)
    rocw, _ = merged_areas([r[0] for r in runs], [r[1] for r in runs], [r[2] for r in runs], roc=True, pr=False)
    torch.testing.assert_close(rocw[0], binary_auroc(X, T, weight=W).double(), rtol=1e-12, atol=1e-12)
