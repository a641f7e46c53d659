"""Edit distance and error totals shared by the word-level text metrics (parity: functional/text/helper.py)."""

from typing import List, Tuple, Union

import torch

from torcheval_amd.ops import native_loaded


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
