"""Throughput, functional API (parity: functional/aggregation/throughput.py)."""

import torch

__all__ = ["throughput"]


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
