"""Sample-sharded AUROC / AUPRC with ROCm-resident shards: two gloo ranks on one GPU, each
running the K3a sort + K3 scan with shard offsets on its received key range."""

import pytest
import torch

from torcheval_amd.metrics.functional import binary_auprc, binary_auroc
from torcheval_amd.utils.test_utils.dist_pool import run_distributed

pytestmark = pytest.mark.gpu


def _data(ws):
    g = torch.Generator().manual_seed(5)
    xs = [(torch.randint(0, 500, (n,), generator=g).float() / 500) for n in (30_000, 70_001)[:ws]]
    ts = [torch.randint(0, 2, (x.numel(),), generator=g) for x in xs]
    return xs, ts


def _job(rank, world_size):
    from torcheval_amd.parallel.dist_auc import distributed_binary_areas

    xs, ts = _data(world_size)
    roc, pr = distributed_binary_areas(xs[rank].cuda(), ts[rank].cuda())
    assert roc.is_cuda
    return float(roc), float(pr)


def test_sharded_auc_on_gpu():
    xs, ts = _data(2)
    want_roc = float(binary_auroc(torch.cat(xs), torch.cat(ts)))
    want_pr = float(binary_auprc(torch.cat(xs), torch.cat(ts)))
    for roc, pr in run_distributed(_job, 2):
        assert abs(roc - want_roc) < 1e-9
        assert abs(pr - want_pr) < 1e-6
