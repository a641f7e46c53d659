"""Word error rate, functional API (parity: functional/text/word_error_rate.py)."""

from typing import List, Tuple, Union

import torch

from torcheval_amd.metrics.functional.text.helper import _get_errors_and_totals, _text_pair_check

__all__ = ["word_error_rate"]


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
