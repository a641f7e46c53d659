"""BLEU score, functional API (parity: functional/text/bleu.py)."""

from collections import Counter
from typing import Optional, Sequence, Tuple, Union

import torch

from torcheval_amd.ops import native_loaded

__all__ = ["bleu_score"]


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
