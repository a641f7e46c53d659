"""Class-dimension sharded sync (``torcheval_amd.parallel.class_shard``) on a gloo world: the
sharded results must equal the single-process compute over every rank's data."""

import unittest

import torch

from torcheval_amd.metrics import MulticlassBinnedAUPRC, MulticlassConfusionMatrix, MultilabelBinnedAUPRC
from torcheval_amd.utils.test_utils.dist_pool import run_distributed


def _data(rank: int, C: int, seed: int):
    g = torch.Generator().manual_seed(seed * 100 + rank)
    n = 200 + 37 * rank
    return torch.rand(n, C, generator=g).softmax(-1), torch.randint(0, C, (n,), generator=g), \
        torch.randint(0, 2, (n, C), generator=g)


def _job(rank: int, ws: int, C: int, normalize):
    from torcheval_amd.parallel import class_sharded_compute, sharded_confusion_matrix

    x, y, yl = _data(rank, C, 1)
    cm = MulticlassConfusionMatrix(C, normalize=normalize).update(x, y)
    ap = MulticlassBinnedAUPRC(num_classes=C, threshold=20, average=None).update(x, y)
    ml = MultilabelBinnedAUPRC(num_labels=C, threshold=10).update(x, yl)
    shard = sharded_confusion_matrix(cm)
    return (shard.start, shard.stop, shard.rows, class_sharded_compute(cm),
            class_sharded_compute(ap), class_sharded_compute(ml))


class TestClassShard(unittest.TestCase):
    def _check(self, ws: int, C: int, normalize) -> None:
        ref_cm = MulticlassConfusionMatrix(C, normalize=normalize)
        ref_ap = MulticlassBinnedAUPRC(num_classes=C, threshold=20, average=None)
        ref_ml = MultilabelBinnedAUPRC(num_labels=C, threshold=10)
        for r in range(ws):
            x, y, yl = _data(r, C, 1)
            ref_cm.update(x, y)
            ref_ap.update(x, y)
            ref_ml.update(x, yl)
        want_cm, want_ap, want_ml = ref_cm.compute(), ref_ap.compute(), ref_ml.compute()
        out = run_distributed(_job, ws, C, normalize)
        covered = 0
        for start, stop, rows, cm, ap, ml in out:
            torch.testing.assert_close(rows, want_cm[start:stop])
            covered += stop - start
            torch.testing.assert_close(cm, want_cm)
            torch.testing.assert_close(ap, want_ap)
            torch.testing.assert_close(ml, want_ml)
        self.assertEqual(covered, C)

    def test_ws2_even(self) -> None:
        self._check(2, 8, None)

    def test_ws3_uneven_pred(self) -> None:
        self._check(3, 7, "pred")

    def test_ws3_true_all(self) -> None:
        self._check(3, 5, "true")
        self._check(3, 5, "all")

    def test_fewer_classes_than_ranks(self) -> None:
        self._check(3, 2, None)


if __name__ == "__main__":
    unittest.main()
