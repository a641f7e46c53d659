"""Binary normalized entropy, functional API
(parity: functional/classification/binary_normalized_entropy.py:14-152).

NE = mean weighted BCE / entropy of the (weighted) base positive rate, per task, float64.
ROCm tensors use the fused K6 row-reduction kernel (BCE or BCE-with-logits, weighted counts
and the probability-range check in one pass; the range check is a device flag instead of
the reference's host-synchronising ``input.max()/min()``).
"""

import struct
from typing import Optional, Tuple

import torch

from torcheval_amd.metrics.functional.tensor_utils import _require_samples
import torch.nn.functional as F

from torcheval_amd.ops import use_native
from torcheval_amd.ops.hostread import read_int, read_ints


@torch.inference_mode()
def binary_normalized_entropy(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    weight: Optional[torch.Tensor] = None,
    num_tasks: int = 1,
    from_logits: bool = False,
) -> torch.Tensor:
    """Normalized (binary) cross entropy of ``[n]`` / ``[num_tasks, n]`` predictions.
    Class version: ``BinaryNormalizedEntropy``."""
    cross_entropy, num_positive, num_examples = _binary_normalized_entropy_update(
        input, target, from_logits, num_tasks, weight
    )
    cross_entropy = cross_entropy / num_examples
    baseline_entropy = _baseline_update(num_positive, num_examples)
    return (cross_entropy / baseline_entropy).double()


def _binary_normalized_entropy_update(
    input: torch.Tensor,
    target: torch.Tensor,
    from_logits: bool,
    num_tasks: int,
    weight: Optional[torch.Tensor] = None,
    err: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(sum of weighted BCE, weighted positives, weighted examples) per task (float64).

    On the GPU path a range violation is recorded in ``err`` (int32[1]) when given (checked
    later by the caller); otherwise it is checked immediately (one sync)."""
    _require_samples(input.numel(), "binary_normalized_entropy")
    _ne_shape_check(input, target, num_tasks, weight)
    if use_native(input) and target.is_cuda and (weight is None or weight.is_cuda):
        from torcheval_amd.ops.reductions import ne_sums

        out, flag = ne_sums(input, target, weight, from_logits, err)
        if err is None and not from_logits:
            _raise_range(flag, input)
        if input.ndim == 1:
            return out[0, 0], out[0, 1], out[0, 2]
        return out[:, 0], out[:, 1], out[:, 2]
    _ne_range_check(input, from_logits)
    return _update(input, target, from_logits, weight)


def _update(
    input: torch.Tensor,
    target: torch.Tensor,
    from_logits: bool,
    weight: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    target_f = target.to(input.dtype) if not target.is_floating_point() else target
    if from_logits:
        ce = F.binary_cross_entropy_with_logits(input, target_f, weight, reduction="none")
    else:
        ce = F.binary_cross_entropy(input, target_f, weight, reduction="none")
    cross_entropy = ce.sum(dim=-1)
    w = torch.ones_like(target_f) if weight is None else weight
    num_examples = w.sum(dim=-1).double()
    num_positive = (w * target_f).sum(dim=-1).double()
    return cross_entropy, num_positive, num_examples


def _baseline_update(num_positive: torch.Tensor, num_examples: torch.Tensor) -> torch.Tensor:
    eps = torch.finfo(torch.float64).eps
    rate = torch.clamp(num_positive / num_examples, min=eps, max=1 - eps)
    return -rate * torch.log(rate) - (1 - rate) * torch.log(1 - rate)


def _raise_range(flag: torch.Tensor, input: torch.Tensor) -> None:
    if read_int(flag) != 0:
        _ne_range_check(input, False)


def _ne_shape_check(
    input: torch.Tensor,
    target: torch.Tensor,
    num_tasks: int,
    weight: Optional[torch.Tensor] = None,
) -> None:
    if input.shape != target.shape:
        raise ValueError(
            f"`input` shape ({input.shape}) is different from `target` shape ({target.shape})"
        )
    if weight is not None and input.shape != weight.shape:
        raise ValueError(
            f"`weight` shape ({weight.shape}) is different from `input` shape ({input.shape})"
        )
    if num_tasks == 1:
        if len(input.shape) > 1:
            raise ValueError(
                f"`num_tasks = 1`, `input` is expected to be one-dimensional tensor, but got shape ({input.shape})."
            )
    elif len(input.shape) == 1 or input.shape[0] != num_tasks:
        raise ValueError(
            f"`num_tasks = {num_tasks}`, `input`'s shape is expected to be ({num_tasks}, num_samples), but got shape ({input.shape})."
        )


def _ne_device_error(err: torch.Tensor, from_logits: bool, dtype: torch.dtype) -> None:
    """Raise a range violation that GPU class updates recorded in ``err`` (int32[6]: flag, pad,
    then the kernel's order-preserving u64 keys of max / complemented min of the inputs) with
    the reference's message.  The range is over every update since the last check, which is
    the failing batch's own range when one update was bad (the reference raises at that
    update)."""
    vals = read_ints(err)
    if vals[0] == 0:
        return
    err.zero_()
    mask = (1 << 64) - 1
    # words 2-5: two little-endian u64 keys (max, complemented min)
    kmax = (vals[2] & 0xFFFFFFFF) | ((vals[3] & 0xFFFFFFFF) << 32)
    kmin = (vals[4] & 0xFFFFFFFF) | ((vals[5] & 0xFFFFFFFF) << 32)

    def decode(key: int) -> float:
        u = key & ~(1 << 63) if key >> 63 else ~key & mask
        return struct.unpack("<d", u.to_bytes(8, "little"))[0]

    if kmax == 0 or kmin == 0:  # no range recorded: report the violation without one
        _ne_range_check(torch.tensor([2.0]), from_logits)
        return
    _ne_range_check(torch.tensor([decode(~kmin & mask), decode(kmax)], dtype=dtype), from_logits)


def _ne_range_check(input: torch.Tensor, from_logits: bool) -> None:
    if from_logits or input.numel() == 0:
        return
    input_max, input_min = input.max(), input.min()
    if input_max > 1.0 or input_min < 0.0:
        raise ValueError(
            f"`from_logits`={from_logits}, `input` should be probability in range [0., 1.], but got `input` ranging",
            f"from {input_min} to {input_max}.",
            "Please set `from_logits = True` or convert `input` into valid probability value. ",
        )


def _ne_input_check(
    input: torch.Tensor,
    target: torch.Tensor,
    from_logits: bool,
    num_tasks: int,
    weight: Optional[torch.Tensor] = None,
) -> None:
    _ne_shape_check(input, target, num_tasks, weight)
    _ne_range_check(input, from_logits)
