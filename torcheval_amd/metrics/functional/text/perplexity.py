"""Perplexity, functional API (parity: functional/text/perplexity.py); K7 fused log-softmax gather on ROCm."""

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from torcheval_amd.metrics.functional.tensor_utils import _require_samples
from torcheval_amd.ops import use_native
from torcheval_amd.ops.hostread import read_int

__all__ = ["perplexity"]


@torch.inference_mode()
def perplexity(input: torch.Tensor, target: torch.Tensor, ignore_index: Optional[int] = None) -> torch.Tensor:
    """exp(mean token negative log-likelihood) of [B, S, V] logits vs [B, S] targets (float64).
    Class version: ``Perplexity``."""
    if use_native(input) and target.is_cuda:
        # K7 records out-of-range targets on the device; the exp / divide is enqueued before the
        # flag is read, so the host read waits once for everything instead of gating the launch
        flag = torch.zeros(1, dtype=torch.int32, device=input.device)
        sum_log_probs, num_total = _perplexity_update(input, target, ignore_index, err=flag)
        out = _perplexity_compute(sum_log_probs, num_total)
        if read_int(flag) != 0:
            _perplexity_label_check(input, target, ignore_index)
        return out
    sum_log_probs, num_total = _perplexity_update(input, target, ignore_index)
    return _perplexity_compute(sum_log_probs, num_total)


def _perplexity_update(
    input: torch.Tensor,
    target: torch.Tensor,
    ignore_index: Optional[int] = None,
    err: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    _perplexity_shape_check(input, target)
    _require_samples(target.numel(), "perplexity")
    logits = input.reshape(-1, input.shape[-1])
    tgt = target.reshape(-1)
    if use_native(input) and tgt.is_cuda and input.dtype in (torch.float32, torch.bfloat16, torch.float16):
        from torcheval_amd.ops import native

        if logits.stride(-1) != 1:
            logits = logits.contiguous()
        out = torch.zeros(2, dtype=torch.float64, device=input.device)
        flag = err if err is not None else torch.zeros(1, dtype=torch.int32, device=input.device)
        from torcheval_amd.config import config

        native().perplexity_sums(logits, tgt, ignore_index, out, flag, config.deterministic)
        if err is None and read_int(flag) != 0:
            _perplexity_label_check(input, target, ignore_index)
        return out[0], out[1]
    _perplexity_label_check(input, target, ignore_index)
    if ignore_index is not None:
        keep = tgt.ne(ignore_index)
        logits, tgt = logits[keep], tgt[keep]
    logp = F.log_softmax(logits.float() if logits.dtype in (torch.float16, torch.bfloat16) else logits, dim=1)
    nll = -logp.gather(1, tgt.unsqueeze(1)).sum()
    return nll, torch.tensor(tgt.size(0), device=tgt.device)


def _perplexity_compute(sum_log_probs: torch.Tensor, num_total: torch.Tensor) -> torch.Tensor:
    return torch.exp(sum_log_probs / num_total).double()


def _perplexity_shape_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if target.ndim != 2:
        raise ValueError(f"target should be a two-dimensional tensor, got shape {target.shape}.")
    if input.ndim != 3:
        raise ValueError(f"input should be a three-dimensional tensor, got shape {input.shape}.")
    if input.size(0) != target.size(0):
        raise ValueError(
            "The `input` and `target` should have the same first dimension (i.e., batch size), "
            f"got shapes {input.shape} and {target.shape} instead."
        )
    if input.size(1) != target.size(1):
        raise ValueError(
            "The `input` and `target` should have the same second dimension (i.e., sequence length), "
            f"got shapes {input.shape} and {target.shape} instead."
        )


def _perplexity_label_check(input: torch.Tensor, target: torch.Tensor, ignore_index: Optional[int]) -> None:
    t = target[target.ne(ignore_index)] if ignore_index else target
    if t.numel() and input.size(2) <= torch.max(t):
        raise ValueError(
            "Class labels in `target` tensor cannot be larger than vocab_size minus one, "
            f"got vocab size of {input.size(2)} and target label of {int(torch.max(t))}."
        )


def _perplexity_input_check(input: torch.Tensor, target: torch.Tensor, ignore_index: Optional[int] = None) -> None:
    _perplexity_shape_check(input, target)
    _perplexity_label_check(input, target, ignore_index)
