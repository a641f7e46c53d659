"""Sample-sharded exact AUROC / AUPRC (``torcheval_amd.parallel.dist_auc``) on a real gloo world:
every rank holds a different, unevenly sized shard; the result must equal the single-process
``binary_auroc`` / ``binary_auprc`` of the concatenation (ties across ranks, weights, an empty
shard, a one-class shard)."""

import unittest

import torch

from torcheval_amd.metrics.functional import binary_auprc, binary_auroc
from torcheval_amd.utils.test_utils.dist_pool import run_distributed


def _case(seed: int, ws: int, ties: bool, weighted: bool, empty_rank: int):
    g = torch.Generator().manual_seed(seed)
    sizes = [int(torch.randint(50, 400, (1,), generator=g)) for _ in range(ws)]
    if empty_rank >= 0:
        sizes[empty_rank] = 0
    xs, ts, wsl = [], [], []
    for n in sizes:
        x = (torch.randint(0, 12, (n,), generator=g).float() / 12) if ties else torch.rand(n, generator=g)
        xs.append(x)
        ts.append(torch.randint(0, 2, (n,), generator=g))
        wsl.append(torch.rand(n, generator=g) if weighted else None)
    return xs, ts, wsl


def _job(rank: int, world_size: int, seed: int, ties: bool, weighted: bool, empty_rank: int):
    from torcheval_amd.parallel.dist_auc import distributed_binary_areas

    xs, ts, wsl = _case(seed, world_size, ties, weighted, empty_rank)
    roc, pr = distributed_binary_areas(xs[rank], ts[rank], wsl[rank], samples_per_rank=16)
    return float(roc), float(pr)


class TestDistributedAUC(unittest.TestCase):
    def _check(self, ws: int, seed: int, ties: bool, weighted: bool, empty_rank: int = -1) -> None:
        xs, ts, wsl = _case(seed, ws, ties, weighted, empty_rank)
        x, t = torch.cat(xs), torch.cat(ts)
        w = torch.cat(wsl) if weighted else None
        want_roc = float(binary_auroc(x, t, weight=w)) if weighted else float(binary_auroc(x, t))
        want_pr = float(binary_auprc(x, t))
        out = run_distributed(_job, ws, seed, ties, weighted, empty_rank)
        for roc, pr in out:
            self.assertAlmostEqual(roc, want_roc, places=10)
            if not weighted:  # binary_auprc has no weight argument (reference API)
                self.assertAlmostEqual(pr, want_pr, places=6)  # binary_auprc returns fp32
        self.assertEqual(len({o for o in out}), 1)  # every rank agrees exactly

    def test_ws2_random(self) -> None:
        self._check(2, 0, ties=False, weighted=False)

    def test_ws2_ties_cross_rank(self) -> None:
        self._check(2, 1, ties=True, weighted=False)

    def test_ws3_weighted_ties(self) -> None:
        self._check(3, 2, ties=True, weighted=True)

    def test_ws3_empty_shard(self) -> None:
        self._check(3, 3, ties=True, weighted=False, empty_rank=1)

    def test_single_process(self) -> None:
        from torcheval_amd.parallel.dist_auc import distributed_binary_auprc, distributed_binary_auroc

        xs, ts, _ = _case(4, 1, True, False, -1)
        torch.testing.assert_close(distributed_binary_auroc(xs[0], ts[0]), binary_auroc(xs[0], ts[0]).double())
        torch.testing.assert_close(distributed_binary_auprc(xs[0], ts[0]).float(), binary_auprc(xs[0], ts[0]))
        # one-class input: AUROC 0.5, AUPRC 0 (single-device conventions)
        ones = torch.ones(10, dtype=torch.long)
        self.assertEqual(float(distributed_binary_auroc(torch.rand(10), ones)), float(binary_auroc(torch.rand(10), ones)))


if __name__ == "__main__":
    unittest.main()


def _metric_job(rank: int, world_size: int):
    from torcheval_amd.metrics import BinaryAUPRC, BinaryAUROC
    from torcheval_amd.parallel import sharded_compute

    xs, ts, wsl = _case(11, world_size, True, True, -1)
    m = BinaryAUROC()
    if rank == 0:  # one weighted rank, one unweighted rank, two updates each
        m.update(xs[rank][:40], ts[rank][:40], wsl[rank][:40]).update(xs[rank][40:], ts[rank][40:], wsl[rank][40:])
    else:
        m.update(xs[rank][:40], ts[rank][:40]).update(xs[rank][40:], ts[rank][40:])
    p = BinaryAUPRC()
    if rank != 1:  # rank 1 never updates
        p.update(xs[rank], ts[rank])
    return float(sharded_compute(m)), float(sharded_compute(p))


class TestShardedCompute(unittest.TestCase):
    def test_metric_integration(self) -> None:
        xs, ts, wsl = _case(11, 2, True, True, -1)
        w = torch.cat([wsl[0], torch.ones(len(xs[1]))])
        want_roc = float(binary_auroc(torch.cat(xs), torch.cat(ts), weight=w))
        want_pr = float(binary_auprc(xs[0], ts[0]))
        for roc, pr in run_distributed(_metric_job, 2):
            self.assertAlmostEqual(roc, want_roc, places=10)
            self.assertAlmostEqual(pr, want_pr, places=6)
