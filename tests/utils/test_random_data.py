"""Synthetic data generators (parity: reference tests/utils/test_random_data.py): shapes with
the update / task dims squeezed when 1, value ranges, target alphabets, threshold invariants."""

import pytest
import torch

from torcheval_amd.utils import random_data as rd


@pytest.mark.parametrize(
    "updates,tasks,batch,shape",
    [(1, 1, 8, (8,)), (1, 3, 8, (3, 8)), (4, 1, 8, (4, 8)), (4, 3, 8, (4, 3, 8))],
)
def test_binary_shapes_and_ranges(updates, tasks, batch, shape):
    x, y = rd.get_rand_data_binary(updates, tasks, batch)
    assert x.shape == shape and y.shape == shape
    assert x.dtype == torch.float32 and y.dtype == torch.int64
    assert bool(((x >= 0) & (x < 1)).all()) and set(y.unique().tolist()) <= {0, 1}


@pytest.mark.parametrize("updates,classes,batch", [(1, 4, 16), (5, 3, 16)])
def test_multiclass_shapes_and_ranges(updates, classes, batch):
    x, y = rd.get_rand_data_multiclass(updates, classes, batch)
    exp_x = (batch, classes) if updates == 1 else (updates, batch, classes)
    assert x.shape == exp_x and y.shape == exp_x[:-1]
    assert int(y.min()) >= 0 and int(y.max()) < classes


@pytest.mark.parametrize("updates,labels,batch", [(1, 4, 16), (5, 3, 16)])
def test_multilabel_shapes_and_ranges(updates, labels, batch):
    x, y = rd.get_rand_data_multilabel(updates, labels, batch)
    exp = (batch, labels) if updates == 1 else (updates, batch, labels)
    assert x.shape == exp and y.shape == exp
    assert set(y.unique().tolist()) <= {0, 1}


@pytest.mark.parametrize("bins", [2, 5, 50])
def test_binned_thresholds_sorted_unique_with_endpoints(bins):
    x, y, thr = rd.get_rand_data_binned_binary(3, 2, 10, bins)
    assert x.shape == (3, 2, 10) and y.shape == (3, 2, 10)
    assert float(thr[0]) == 0.0 and float(thr[-1]) == 1.0
    assert bool((thr[1:] > thr[:-1]).all()) and thr.numel() <= bins


def test_seeded_reproducible():
    torch.manual_seed(5)
    a = rd.get_rand_data_multiclass(2, 3, 4)
    torch.manual_seed(5)
    b = rd.get_rand_data_multiclass(2, 3, 4)
    assert all(torch.equal(p, q) for p, q in zip(a, b))


@pytest.mark.gpu
def test_device_placement_gpu():
    dev = torch.device("cuda", 0)
    for x in (*rd.get_rand_data_binary(2, 2, 4, device=dev), *rd.get_rand_data_binned_binary(1, 1, 4, 5, device=dev)):
        assert x.device == dev
