"""Aggregation metrics, functional API (parity: functional/aggregation/{auc,mean,sum,throughput}.py)."""

from typing import Tuple, Union

import torch

__all__ = ["auc", "mean", "sum", "throughput"]
__doc_name__ = "Aggregation Metrics"

_builtin_sum = sum


def _auc_compute(x: torch.Tensor, y: torch.Tensor, reorder: bool = False) -> torch.Tensor:
    if x.numel() == 0 or y.numel() == 0:
        return torch.tensor([])
    if x.ndim == 1:
        x = x.unsqueeze(0)
    if y.ndim == 1:
        y = y.unsqueeze(0)
    if reorder:
        x, idx = torch.sort(x, dim=1, stable=True)
        y = y.gather(1, idx)
    return torch.trapz(y, x)


def _auc_update_input_check(x: torch.Tensor, y: torch.Tensor, n_tasks: int = 1) -> None:
    size_x, size_y = x.size(), y.size()
    if x.ndim == 1:
        x = x.unsqueeze(0)
    if y.ndim == 1:
        y = y.unsqueeze(0)
    if x.numel() == 0 or y.numel() == 0:
        raise ValueError(
            f"The `x` and `y` should have atleast 1 element, got shapes {size_x} and {size_y}."
        )
    if x.size() != y.size():
        raise ValueError(
            f"Expected the same shape in `x` and `y` tensor but got shapes {size_x} and {size_y}."
        )
    if x.size(0) != n_tasks or y.size(0) != n_tasks:
        raise ValueError(
            f"Expected `x` dim_1={x.size(0)} and `y` dim_1={y.size(0)} have first dimension equals to n_tasks={n_tasks}."
        )


def auc(x: torch.Tensor, y: torch.Tensor, reorder: bool = False) -> torch.Tensor:
    """Trapezoidal area under the curve y(x) per task (``[n]`` or ``[n_tasks, n]``).
    Class version: ``torcheval_amd.metrics.AUC``."""
    n_tasks = x.size(0) if x.ndim > 1 else 1
    _auc_update_input_check(x, y, n_tasks)
    return _auc_compute(x, y, reorder)


def _mean_update(
    input: torch.Tensor, weight: Union[float, int, torch.Tensor]
) -> Tuple[torch.Tensor, torch.Tensor]:
    if isinstance(weight, (float, int)):
        return weight * torch.sum(input), torch.tensor(float(weight) * torch.numel(input), device=input.device)
    if isinstance(weight, torch.Tensor) and input.size() == weight.size():
        return torch.sum(weight * input), torch.sum(weight)
    raise ValueError(
        "Weight must be either a float value or a tensor that matches the input tensor size. "
        f"Got {weight} instead."
    )


def _mean_compute(input: torch.Tensor, weight: Union[float, int, torch.Tensor]) -> torch.Tensor:
    weighted_sum, weights = _mean_update(input, weight)
    return weighted_sum / weights


@torch.inference_mode()
def mean(input: torch.Tensor, weight: Union[float, int, torch.Tensor] = 1.0) -> torch.Tensor:
    """Weighted mean.  Class version: ``torcheval_amd.metrics.Mean``."""
    return _mean_compute(input, weight)


def _sum_update(input: torch.Tensor, weight: Union[float, int, torch.Tensor]) -> torch.Tensor:
    if isinstance(weight, (float, int)) or (
        isinstance(weight, torch.Tensor) and input.size() == weight.size()
    ):
        return (input * weight).sum()
    raise ValueError(
        "Weight must be either a float value or an int value or a tensor that matches the input tensor size. "
        f"Got {weight} instead."
    )


@torch.inference_mode()
def sum(input: torch.Tensor, weight: Union[float, torch.Tensor] = 1.0) -> torch.Tensor:  # noqa: A001
    """Weighted sum.  Class version: ``torcheval_amd.metrics.Sum``."""
    return _sum_update(input, weight)


def _throughput_compute(num_processed: int, elapsed_time_sec: float) -> torch.Tensor:
    if num_processed < 0:
        raise ValueError(
            f"Expected num_processed to be a non-negative number, but received {num_processed}."
        )
    if elapsed_time_sec <= 0:
        raise ValueError(
            f"Expected elapsed_time_sec to be a positive number, but received {elapsed_time_sec}."
        )
    return torch.tensor(num_processed / elapsed_time_sec)


@torch.inference_mode()
def throughput(num_processed: int = 0, elapsed_time_sec: float = 0.0) -> torch.Tensor:
    """Items per second.  Class version: ``torcheval_amd.metrics.Throughput``."""
    return _throughput_compute(num_processed, elapsed_time_sec)
