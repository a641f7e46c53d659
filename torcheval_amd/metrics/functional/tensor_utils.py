"""Small tensor helpers (parity: functional/tensor_utils.py:12-33)."""

import weakref
from typing import Dict, List, Tuple, Union

import torch

# Threshold tensors known to be sorted and inside [0, 1]: ints -> cached linspace, validated
# lists, and user tensors after their first (single-sync) check.  Keyed by id with a weak
# value so a freed tensor's id can never alias a validated one.
_VALIDATED: "weakref.WeakValueDictionary[int, torch.Tensor]" = weakref.WeakValueDictionary()
_LINSPACE: Dict[Tuple[int, str], torch.Tensor] = {}
# the cached linspace(0, 1, n) tensors themselves: the K4 kernels may bin them arithmetically
_UNIFORM: "weakref.WeakValueDictionary[int, torch.Tensor]" = weakref.WeakValueDictionary()


def _is_uniform_linspace(t: torch.Tensor) -> bool:
    """True iff ``t`` is (the very tensor) ``linspace(0, 1, n)`` made from an int threshold.
    (A speed hint only: under torch.compile the weak-reference lookup is skipped.)"""
    from torch.compiler import is_compiling

    if is_compiling():
        return False
    return _UNIFORM.get(id(t)) is t


def _move_threshold(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    """``t`` on ``device``, keeping its validated / uniform-linspace markers."""
    if t.device == device:
        return t
    moved = t.to(device)
    if _VALIDATED.get(id(t)) is t:
        _VALIDATED[id(moved)] = moved
    if _UNIFORM.get(id(t)) is t:
        _UNIFORM[id(moved)] = moved
    return moved


def _riemann_integral(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Left Riemann sum of y over the (descending) x grid: -sum((x[1:] - x[:-1]) * y[:-1])."""
    return -torch.sum((x[1:] - x[:-1]) * y[:-1])


def _create_threshold_tensor(
    threshold: Union[int, List[float], torch.Tensor], device: torch.device
) -> torch.Tensor:
    """An int n becomes ``linspace(0, 1, n)``; a list becomes a tensor; tensors pass through.

    Int thresholds are cached per (n, device) - no per-call linspace launch - and, like lists
    (checked on the host before the copy), are marked valid so ``_threshold_check`` skips the
    device round trip the reference pays on every call."""
    if isinstance(threshold, int):
        key = (threshold, str(torch.device(device)))
        t = _LINSPACE.get(key)
        if t is None:
            t = torch.linspace(0, 1.0, threshold, device=device)
            _LINSPACE[key] = t
            _VALIDATED[id(t)] = t
            if threshold >= 2:
                _ENDPOINTS_OK[id(t)] = t
                _UNIFORM[id(t)] = t
        return t
    if isinstance(threshold, list):
        _check_host(threshold)
        t = torch.tensor(threshold, device=device)
        _VALIDATED[id(t)] = t
        if threshold and threshold[0] == 0 and threshold[-1] == 1:
            _ENDPOINTS_OK[id(t)] = t
        return t
    return threshold


def _check_host(values: List[float]) -> None:
    if any(b < a for a, b in zip(values, values[1:])):
        raise ValueError("The `threshold` should be a sorted tensor.")
    if any(v < 0.0 or v > 1.0 for v in values):
        raise ValueError("The values in `threshold` should be in the range of [0, 1].")


_ENDPOINTS_OK: "weakref.WeakValueDictionary[int, torch.Tensor]" = weakref.WeakValueDictionary()


def _threshold_check(threshold: torch.Tensor, endpoints: bool = False) -> None:
    """Sorted and inside [0, 1] (and, with ``endpoints``, starting at 0 and ending at 1), with
    the reference's messages - one host sync for an unseen tensor instead of up to four."""
    known = _VALIDATED.get(id(threshold)) is threshold
    ends = _ENDPOINTS_OK.get(id(threshold)) is threshold
    if known and (ends or not endpoints):
        return
    checks = [(torch.diff(threshold) < 0.0).any(), ((threshold < 0.0) | (threshold > 1.0)).any()]
    if endpoints:
        checks += [threshold[0] != 0, threshold[-1] != 1]
    flags = torch.stack(checks).tolist()
    if flags[0]:
        raise ValueError("The `threshold` should be a sorted tensor.")
    if flags[1]:
        raise ValueError("The values in `threshold` should be in the range of [0, 1].")
    if endpoints and flags[2]:
        raise ValueError("First value in `threshold` should be 0.")
    if endpoints and flags[3]:
        raise ValueError("Last value in `threshold` should be 1.")
    _VALIDATED[id(threshold)] = threshold
    if endpoints:
        _ENDPOINTS_OK[id(threshold)] = threshold


def _require_samples(n: int, name: str) -> None:
    """The reference crashes inside TorchScript / ``torch.max`` on an empty input
    (RuntimeError with an internal message); raise the same exception type, with a clear one."""
    if n == 0:
        raise RuntimeError(f"{name}: the input has no samples (the metric is undefined on an empty input).")
