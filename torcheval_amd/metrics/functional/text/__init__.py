"""Text metrics, functional API (parity: functional/text/*.py).

* BLEU and the word-level edit-distance metrics (WER / WIL / WIP) run in the native C++
  runtime (csrc/runtime/text.cpp: interned tokens, two-row Levenshtein DP, hashed n-gram
  counters, GIL released) instead of pure-Python loops; results are identical.
* Perplexity runs the fused K7 HIP kernel on ROCm tensors (online log-sum-exp + target
  gather); the reference materialises an (N x N) probability gather (perplexity.py:102).
"""

from collections import Counter
from typing import List, Optional, Sequence, Tuple, Union

import torch

from torcheval_amd.metrics.functional.tensor_utils import _require_samples
import torch.nn.functional as F

from torcheval_amd.ops import native_loaded, use_native

__all__ = [
    "bleu_score",
    "perplexity",
    "word_error_rate",
    "word_information_lost",
    "word_information_preserved",
]
__doc_name__ = "Text Metrics"


# ----------------------------------------------------------------------------- edit distance
def _edit_distance(prediction_tokens: List[str], reference_tokens: List[str]) -> int:
    """Word-level Levenshtein distance (pure-Python fallback; the runtime does this in C++)."""
    n, m = len(prediction_tokens), len(reference_tokens)
    prev = list(range(m + 1))
    for i in range(1, n + 1):
        cur = [i] + [0] * m
        for j in range(1, m + 1):
            if prediction_tokens[i - 1] == reference_tokens[j - 1]:
                cur[j] = prev[j - 1]
            else:
                cur[j] = min(prev[j], cur[j - 1], prev[j - 1]) + 1
        prev = cur
    return prev[m]


def _get_errors_and_totals(
    input: Union[str, List[str]], target: Union[str, List[str]]
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """errors, max_total, target_total, input_total over sentence pairs (float64 CPU tensors)."""
    if isinstance(input, str):
        input = [input]
    if isinstance(target, str):
        target = [target]
    ins = [s.split() for s in input]
    tgs = [s.split() for s in target]
    if native_loaded():
        from torcheval_amd.ops import native

        e, mx, tt, it = native().text_errors_and_totals(ins, tgs)
    else:
        e = mx = tt = it = 0.0
        for a, b in zip(ins, tgs):
            e += _edit_distance(a, b)
            tt += len(b)
            it += len(a)
            mx += max(len(a), len(b))
    f64 = torch.float64
    return torch.tensor(e, dtype=f64), torch.tensor(mx, dtype=f64), torch.tensor(tt, dtype=f64), torch.tensor(it, dtype=f64)


def _text_pair_check(input, target) -> None:
    if type(input) != type(target):
        raise ValueError(
            f"input and target should have the same type, got {type(input)} and {type(target)}."
        )
    if type(input) == list and len(input) != len(target):
        raise ValueError(
            f"input and target lists should have the same length, got {len(input)} and {len(target)}"
        )


# ----------------------------------------------------------------------------- WER / WIL / WIP
@torch.inference_mode()
def word_error_rate(input: Union[str, List[str]], target: Union[str, List[str]]) -> torch.Tensor:
    """Word error rate = word edit distance / reference words.  Class: ``WordErrorRate``."""
    errors, total = _word_error_rate_update(input, target)
    return _word_error_rate_compute(errors, total)


def _word_error_rate_update(
    input: Union[str, List[str]], target: Union[str, List[str]]
) -> Tuple[torch.Tensor, torch.Tensor]:
    _text_pair_check(input, target)
    errors, _, target_total, _ = _get_errors_and_totals(input, target)
    return errors, target_total


def _word_error_rate_compute(errors: torch.Tensor, total: torch.Tensor) -> torch.Tensor:
    return errors / total


def _wil_update(
    input: Union[str, List[str]], target: Union[str, List[str]]
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if isinstance(input, str):
        input = [input]
    if isinstance(target, str):
        target = [target]
    assert len(input) == len(target), (
        "Arguments must contain the same number of strings, "
        f"but got len(input)={len(input)} and len(target)={len(target)}"
    )
    errors, max_total, target_total, input_total = _get_errors_and_totals(input, target)
    # (errors - max_total) is the NEGATED number of hits; the square in compute hides the sign
    return errors - max_total, target_total, input_total


def _wil_compute(correct_total: torch.Tensor, target_total: torch.Tensor, preds_total: torch.Tensor) -> torch.Tensor:
    return 1 - correct_total / target_total * (correct_total / preds_total)


@torch.inference_mode()
def word_information_lost(input: Union[str, List[str]], target: Union[str, List[str]]) -> torch.Tensor:
    """Word information lost.  Class: ``WordInformationLost``."""
    return _wil_compute(*_wil_update(input, target))


@torch.inference_mode()
def word_information_preserved(input: Union[str, List[str]], target: Union[str, List[str]]) -> torch.Tensor:
    """Word information preserved.  Class: ``WordInformationPreserved``."""
    return _word_information_preserved_compute(*_word_information_preserved_update(input, target))


def _word_information_preserved_update(
    input: Union[str, List[str]], target: Union[str, List[str]]
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _text_pair_check(input, target)
    errors, max_total, target_total, input_total = _get_errors_and_totals(input, target)
    return max_total - errors, target_total, input_total


def _word_information_preserved_compute(
    correct_total: torch.Tensor, target_total: torch.Tensor, input_total: torch.Tensor
) -> torch.Tensor:
    return correct_total / target_total * (correct_total / input_total)


# ----------------------------------------------------------------------------- BLEU
@torch.inference_mode()
def bleu_score(
    input: Union[str, Sequence[str]],
    target: Sequence[Union[str, Sequence[str]]],
    n_gram: int = 4,
    weights: Optional[torch.Tensor] = None,
    device: Optional[torch.device] = None,
) -> torch.Tensor:
    """Corpus BLEU of candidate translations against one or more references each.
    Class version: ``BLEUScore``."""
    stats = _bleu_score_update(input, target, n_gram, device)
    return _bleu_score_compute(*stats, n_gram, weights)


def _bleu_score_update(
    input: Union[str, Sequence[str]],
    target: Sequence[Union[str, Sequence[str]]],
    n_gram: int,
    device: Optional[torch.device] = None,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    input_ = [input] if isinstance(input, str) else input
    target_ = [[tgt] if isinstance(tgt, str) else tgt for tgt in target]
    if len(input_) != len(target_):
        raise ValueError(
            f"Input and target corpus should have same sizes, but input corpus size = {len(input_)}, target corpus size = {len(target_)} "
        )
    if n_gram not in [1, 2, 3, 4]:
        raise ValueError(f"n_gram should be 1, 2, 3, or 4, got {n_gram}.")
    cands = [c.split() for c in input_]
    refs = [[r.split() for r in rs] for rs in target_]
    if native_loaded():
        from torcheval_amd.ops import native

        in_len, tg_len, matches, possible = native().bleu_counts(cands, refs, n_gram)
    else:
        in_len, tg_len, matches, possible = _bleu_counts_py(cands, refs, n_gram)
    matches_t = torch.tensor(matches, dtype=torch.float32, device=device)
    possible_t = torch.tensor(possible, dtype=torch.float32, device=device)
    if torch.min(possible_t) == 0:
        raise ValueError(f"the input is too short to find all n-gram matches with n_gram={n_gram}")
    return (
        torch.tensor(in_len, device=device),
        torch.tensor(tg_len, device=device),
        matches_t,
        possible_t,
    )


def _get_ngrams(sentence: Sequence[str], n_gram: int) -> Counter:
    if n_gram not in [1, 2, 3, 4]:
        raise ValueError(f"n_gram should be 1, 2, 3, or 4, got {n_gram}.")
    counts: Counter = Counter()
    for n in range(1, n_gram + 1):
        for i in range(len(sentence) - n + 1):
            counts[tuple(sentence[i : i + n])] += 1
    return counts


def _bleu_counts_py(cands, refs, n_gram):
    in_len = tg_len = 0
    matches = [0.0] * n_gram
    possible = [0.0] * n_gram
    for cand, rs in zip(cands, refs):
        in_len += len(cand)
        tg_len += min(len(r) for r in rs)
        ref_counts: Counter = Counter()
        for r in rs:
            ref_counts |= _get_ngrams(r, n_gram)
        overlap = _get_ngrams(cand, n_gram) & ref_counts
        for ng, c in overlap.items():
            matches[len(ng) - 1] += c
        for i in range(n_gram):
            if len(cand) - i > 0:
                possible[i] += len(cand) - i
    return in_len, tg_len, matches, possible


def _bleu_score_compute(
    input_len: torch.Tensor,
    target_len: torch.Tensor,
    matches_by_order: torch.Tensor,
    possible_matches_by_order: torch.Tensor,
    n_gram: int,
    weights: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    if weights is not None and n_gram != weights.size(dim=0):
        raise ValueError(
            f"the length of weights should equal n_gram, got len(weights)={weights.size(dim=0)}, n_gram={n_gram}"
        )
    if weights is None:
        weights = torch.tensor([1 / n_gram] * n_gram, device=matches_by_order.device)
    precisions = matches_by_order / possible_matches_by_order
    geometric_mean = torch.exp(torch.sum(weights.to(precisions.device) * torch.log(precisions)))
    return _calc_brevity_penalty(input_len, target_len) * geometric_mean


def _calc_brevity_penalty(input_len: torch.Tensor, target_len: torch.Tensor) -> torch.Tensor:
    if input_len > target_len:
        return torch.tensor(1.0, device=input_len.device)
    return torch.exp(1 - target_len / input_len)


# ----------------------------------------------------------------------------- perplexity
@torch.inference_mode()
def perplexity(input: torch.Tensor, target: torch.Tensor, ignore_index: Optional[int] = None) -> torch.Tensor:
    """exp(mean token negative log-likelihood) of [B, S, V] logits vs [B, S] targets (float64).
    Class version: ``Perplexity``."""
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
        if err is None and int(flag.item()) != 0:
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
