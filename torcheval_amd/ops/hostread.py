"""Low-latency host reads of small int32 / int64 device tensors (error flags, curve sizes).

``compute()`` of a metric whose GPU updates validate labels on the device has to read its
error flag on the host before it may return (the reference raises at ``update()`` instead, on
a host-synchronising check).  ``tensor.item()`` pays a D2H copy plus a stream synchronize
(~17 us idle, ~21 us right behind an update kernel on MI355X); ``read_ints`` publishes the
words into pinned, device-mapped host memory from a one-lane kernel and spins on a sequence
word (~7 / ~12.6 us; ``profiles/host_poll_latency_r4.json``), falling back to a blocking
stream synchronize after ``TORCHEVAL_AMD_HOST_POLL_US`` (default 1000; 0 disables the path).
"""
import os
from typing import List

import torch

import torcheval_amd.ops as _ops

_SPIN_US = int(os.environ.get("TORCHEVAL_AMD_HOST_POLL_US", "1000"))
_MAX_WORDS = 14  # tea::kHostReadWords


def _fast(t: torch.Tensor) -> bool:
    words = t.numel() * (2 if t.dtype == torch.int64 else 1)
    return (
        _SPIN_US > 0
        and t.is_cuda
        and t.dtype in (torch.int32, torch.int64)
        and 1 <= words <= _MAX_WORDS
        and t.is_contiguous()
        and not _ops.DISABLE_HIP
        and _ops.native_loaded()
        and not _ops.compiling()
        and not torch.cuda.is_current_stream_capturing()
    )


def read_ints(t: torch.Tensor) -> List[int]:
    """The elements of ``t`` (flattened) as Python ints, after the work queued before this call."""
    if _fast(t):
        if t.dtype == torch.int64:  # little-endian (lo, hi) int32 pairs
            w = _ops.native().read_small_ints(t.reshape(-1).view(torch.int32), _SPIN_US)
            return [(w[2 * i] & 0xFFFFFFFF) | (w[2 * i + 1] << 32) for i in range(len(w) // 2)]
        return list(_ops.native().read_small_ints(t.reshape(-1), _SPIN_US))
    return [int(v) for v in t.reshape(-1).tolist()]


def read_int(t: torch.Tensor) -> int:
    """The first element of ``t`` as a Python int."""
    if t.numel() == 1 and not t.is_cuda:
        return int(t.item())
    if _fast(t):
        return read_ints(t.reshape(-1)[:1])[0]
    return int(t.reshape(-1)[0].item())


def read_int_pair(a: torch.Tensor, b: torch.Tensor) -> "tuple[int, int]":
    """The first elements of ``a`` and ``b`` as Python ints, in ONE host read when both are int32
    device tensors (one publish launch; two ``read_int`` calls pay two)."""
    a1, b1 = a.reshape(-1)[:1], b.reshape(-1)[:1]
    if a1.dtype == torch.int32 and b1.dtype == torch.int32 and a1.device == b1.device and _fast(a1):
        w = _ops.native().read_small_ints_pair(a1, b1, _SPIN_US)
        return int(w[0]), int(w[1])
    return read_int(a), read_int(b)
