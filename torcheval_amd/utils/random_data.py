"""Synthetic data generators (parity with torcheval/utils/random_data.py:12-161).

Shapes follow the reference: ``[num_updates, num_tasks, batch]`` with the update / task
dimensions dropped when they are 1.  Data is generated on the host with torch's global RNG
(so seeded tests reproduce) and then moved to ``device``.
"""

from typing import List, Optional, Tuple

import torch


def _squeezed_shape(num_updates: int, num_tasks: int, batch_size: int) -> List[int]:
    shape = [num_updates, num_tasks, batch_size]
    if num_updates == 1 and num_tasks == 1:
        return [batch_size]
    if num_updates == 1:
        return [num_tasks, batch_size]
    if num_tasks == 1:
        return [num_updates, batch_size]
    return shape


def get_rand_data_binary(
    num_updates: int,
    num_tasks: int,
    batch_size: int,
    device: Optional[torch.device] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Random scores in [0, 1) and {0, 1} targets, shape ``[updates, tasks, batch]`` (squeezed)."""
    shape = _squeezed_shape(num_updates, num_tasks, batch_size)
    input = torch.rand(size=shape)
    targets = torch.randint(low=0, high=2, size=shape)
    device = device or torch.device("cpu")
    return input.to(device), targets.to(device)


def get_rand_data_multiclass(
    num_updates: int,
    num_classes: int,
    batch_size: int,
    device: Optional[torch.device] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Random ``[updates, batch, classes]`` scores and ``[updates, batch]`` class targets."""
    if num_updates == 1:
        input_shape, targets_shape = [batch_size, num_classes], [batch_size]
    else:
        input_shape = [num_updates, batch_size, num_classes]
        targets_shape = [num_updates, batch_size]
    input = torch.rand(size=input_shape)
    targets = torch.randint(low=0, high=num_classes, size=targets_shape)
    device = device or torch.device("cpu")
    return input.to(device), targets.to(device)


def get_rand_data_multilabel(
    num_updates: int,
    num_labels: int,
    batch_size: int,
    device: Optional[torch.device] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Random ``[updates, batch, labels]`` scores and {0, 1} targets of the same shape."""
    shape = [batch_size, num_labels] if num_updates == 1 else [num_updates, batch_size, num_labels]
    input = torch.rand(size=shape)
    targets = torch.randint(low=0, high=2, size=shape)
    device = device or torch.device("cpu")
    return input.to(device), targets.to(device)


def get_rand_data_binned_binary(
    num_updates: int,
    num_tasks: int,
    batch_size: int,
    num_bins: int,
    device: Optional[torch.device] = None,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Binary data plus sorted unique thresholds in [0, 1] that include 0 and 1."""
    device = device or torch.device("cpu")
    input, target = get_rand_data_binary(num_updates, num_tasks, batch_size, device=device)
    threshold = torch.cat([torch.tensor([0.0, 1.0]), torch.rand(num_bins - 2)])
    threshold = torch.unique(torch.sort(threshold).values)
    return input, target, threshold.to(device)
